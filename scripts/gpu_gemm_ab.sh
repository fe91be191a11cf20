# GEMM A/B: parity tests with the variant forced, then interleaved timing.
# usage: VARIANTS=3,7 bash scripts/gpu_gemm_ab.sh
mkdir -p gpurun_out
V=${VARIANTS:-3,7}
for v in ${TV:-${V//,/ }}; do
  MICLIP_GEMM_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_encode.py -x -q -k "gemm or b32 or small" --timeout 120 --timeout-method thread > gpurun_out/ab_test_$v.log 2>&1 || { echo "tests failed for variant $v"; tail -20 gpurun_out/ab_test_$v.log; exit 1; }
  tail -1 gpurun_out/ab_test_$v.log
done
timeout -k 10 200 python scripts/gemm_micro.py 20 ${SHAPES:-qkv,out,fc,proj,long,qkv20k,fc20k} $V > gpurun_out/ab_micro.log 2>&1 || exit $?
cat gpurun_out/ab_micro.log
