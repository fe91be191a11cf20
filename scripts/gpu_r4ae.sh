# r04 ae: all eight x16 blocks loaded ahead of phase 1's DMAs -- op test + micro
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export MICLIP_LIB=ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -rf -x --timeout 120 --timeout-method thread \
  -k "gemm_residual" > gpurun_out/r4ae_ops.log 2>&1 || { tail -30 gpurun_out/r4ae_ops.log; exit 1; }
tail -1 gpurun_out/r4ae_ops.log
timeout -k 10 300 python -u scripts/gemm_micro.py 10 resout500,resproj500 > gpurun_out/r4ae_micro.log 2>&1 || exit $?
cat gpurun_out/r4ae_micro.log
