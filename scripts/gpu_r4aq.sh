# r04 aq: fused-residual x16 loads: blocks 0-1 in the tile's last pair (phase 6), blocks 2-7 ahead of
# the next tile's phase-1 DMAs (none issued behind them) -- op test + micro
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -rf -x --timeout 120 --timeout-method thread \
  -k "gemm_residual" > gpurun_out/r4aq_ops.log 2>&1 || { tail -30 gpurun_out/r4aq_ops.log; exit 1; }
tail -1 gpurun_out/r4aq_ops.log
timeout -k 10 300 python -u scripts/gemm_micro.py 10 resout500,resproj500 > gpurun_out/r4aq_micro.log 2>&1 || exit $?
cat gpurun_out/r4aq_micro.log
