# r04 au: B/32 attention variants once more (interleaved rounds), two passes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/attn_micro.py 20 B/32c > gpurun_out/r4au_attn.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/attn_micro.py 20 B/32c >> gpurun_out/r4au_attn.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4au_attn.log
