# r04 ah: c_fc with stage-ordered QuickGELU + recomputed store offsets, B/32 attention two heads
# per workgroup -- the tests these touch, attention micro (old kernels as A/B), the bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_encode.py -q -rf -x --timeout 200 --timeout-method thread \
  > gpurun_out/r4ah_tests.log 2>&1 || { tail -30 gpurun_out/r4ah_tests.log; exit 1; }
tail -1 gpurun_out/r4ah_tests.log
timeout -k 10 300 python -u scripts/attn_micro.py 10 B/32c > gpurun_out/r4ah_attn.log 2>&1 || exit $?
cat gpurun_out/r4ah_attn.log
LN_FLAGS=1 timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnfc500 0,1 > gpurun_out/r4ah_lnfc.log 2>&1 || exit $?
cat gpurun_out/r4ah_lnfc.log
timeout -k 10 700 python bench.py --steps 20 --warmup 3 --no-parity-mode > gpurun_out/r4ah_bench.log 2> gpurun_out/r4ah_bench.err || exit $?
tail -1 gpurun_out/r4ah_bench.log | cut -c1-400
