# r04 ag: LDS-staged residual_finalize; short attention as its own kernel (occupancy target) +
# the two-heads-per-workgroup A/B variant
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -q -rf -x --timeout 120 --timeout-method thread \
  -k "gemm_residual or attention" > gpurun_out/r4ag_ops.log 2>&1 || { tail -30 gpurun_out/r4ag_ops.log; exit 1; }
tail -1 gpurun_out/r4ag_ops.log
timeout -k 10 300 python -u scripts/attn_micro.py 10 B/32c,text > gpurun_out/r4ag_attn.log 2>&1 || exit $?
cat gpurun_out/r4ag_attn.log
timeout -k 10 300 python -u scripts/gemm_micro.py 10 resout500 > gpurun_out/r4ag_micro.log 2>&1 || exit $?
cat gpurun_out/r4ag_micro.log
mkdir -p gpurun_out/prof4ag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4ag -o micro -- \
  python3 scripts/gemm_micro.py 3 resout500 > gpurun_out/prof4ag/stdout.log 2>&1 || exit $?
grep -h "finalize\|residual_stats" gpurun_out/prof4ag/micro_kernel_stats.csv | cut -c1-200
LN_FLAGS=1 timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnfc500,lnqkv500 0,4,8,12 > gpurun_out/r4ag_lnflags.log 2>&1 || exit $?
cat gpurun_out/r4ag_lnflags.log
LN_FLAGS=1 timeout -k 10 300 python -u scripts/gemm_micro.py 10 fc500,qkv500 0,4,8,12 > gpurun_out/r4ag_plainflags.log 2>&1 || exit $?
cat gpurun_out/r4ag_plainflags.log
