# r04 y: the JPEG pipeline's first-launch and launch sizes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python scripts/jpeg_first_sub.py > gpurun_out/r4y_first_sub.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4y_first_sub.log
