# Mirrored-corpus kernels: rank GPU tests, then scripts/mirror_micro.py timings.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rank.py tests/test_abi.py -q -rf -x --timeout 120 --timeout-method thread > gpurun_out/pytest_rank.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_rank.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/mirror_micro.py 3 > gpurun_out/mirror_micro.log 2>&1
rc=$?; grep -v "^{" gpurun_out/mirror_micro.log | tail -12; [ $rc -eq 0 ] || exit $rc
true
true
