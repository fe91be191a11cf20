# JPEG + preprocess GPU tests, large-batch debug, folder ingest end to end
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_flows.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_jpeg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_jpeg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ingest_debug.py > gpurun_out/ing_dbg.log 2>&1 || exit $?
cat gpurun_out/ing_dbg.log | grep decode
timeout -k 10 400 python -u scripts/ingest_micro.py 8192 > gpurun_out/ingest_micro.log 2>&1 || exit $?
tail -1 gpurun_out/ingest_micro.log
