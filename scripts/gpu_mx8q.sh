# MX-fp8 8-phase kernel: MX op tests + fp8 tower tests, then the MX GEMM micro (8q / pp / 16x16x128 / bf16).
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_encode.py -q -rf -x --timeout 120 --timeout-method thread > gpurun_out/pytest_mx.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_mx.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/gemm_mx_micro.py 5 > gpurun_out/mx_micro.log 2>&1
rc=$?; cat gpurun_out/mx_micro.log | grep -v amdgpu.ids; exit $rc
