# Round 3: the fp32 tower / R@K flow tests first (verbose, prints kept), then
# the whole GPU suite.  Each GPU step has its own limit; a crash or timeout
# (not a plain test failure) ends the script.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rk_flow.py tests/test_gpu_flows.py tests/test_gpu_encode.py -v -s \
  --timeout 300 --timeout-method thread > gpurun_out/r3a_new.log 2>&1
rc=$?
echo "new tests rc=$rc"; grep -E "PASS|FAIL|ERROR|1-cos|flow:|rel err" gpurun_out/r3a_new.log | tail -60
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3a_gpu.log 2>&1
rc=$?
echo "gpu suite rc=$rc"; tail -15 gpurun_out/r3a_gpu.log
exit $rc
