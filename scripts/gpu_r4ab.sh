# r04 ab: residual add fused into out_proj / c_proj (EPI_RES16_BF16) -- op tests, tower tests,
# micro comparison against the unfused pair, then the bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -q -rf -x --timeout 120 --timeout-method thread \
  -k "gemm_residual or residual_stats or gemm_ln" > gpurun_out/r4ab_ops.log 2>&1 || { tail -30 gpurun_out/r4ab_ops.log; exit 1; }
tail -2 gpurun_out/r4ab_ops.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py -q -rf -x --timeout 200 --timeout-method thread \
  -k "lnfold" > gpurun_out/r4ab_enc.log 2>&1 || { tail -30 gpurun_out/r4ab_enc.log; exit 1; }
tail -2 gpurun_out/r4ab_enc.log
timeout -k 10 300 python -u scripts/gemm_micro.py 10 resout500,resproj500,out500,proj500 > gpurun_out/r4ab_micro.log 2>&1 || exit $?
cat gpurun_out/r4ab_micro.log
timeout -k 10 700 python bench.py --steps 20 --warmup 3 --no-parity-mode > gpurun_out/r4ab_bench.log 2> gpurun_out/r4ab_bench.err || exit $?
tail -1 gpurun_out/r4ab_bench.log | cut -c1-600
