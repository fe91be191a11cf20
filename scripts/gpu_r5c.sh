# r05 c: VALU issue rates of the GELU epilogue's instructions; rank pass phase stamps with the
# rolled slab merge; rank micro timings
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5c
timeout -k 10 60 ./scripts/probes/valu_rate > gpurun_out/r5c/valu_rate.log 2>&1 || exit $?
cat gpurun_out/r5c/valu_rate.log
timeout -k 10 120 python -u scripts/rank_stamp.py > gpurun_out/r5c/rank_stamp.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5c/rank_stamp.log
timeout -k 10 180 python -u scripts/rank_micro.py > gpurun_out/r5c/rank_micro.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5c/rank_micro.log
echo done
