# r04: JPEG ingest timing after removing the copy stream's wait on the compute stream
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4f_pytest.log 2>&1 || exit $?
tail -1 gpurun_out/r4f_pytest.log
timeout -k 10 300 python scripts/jpeg_ingest_micro.py > gpurun_out/r4f_jpeg.log 2>&1 || exit $?
tail -1 gpurun_out/r4f_jpeg.log
timeout -k 10 300 python scripts/jpeg_breakdown.py > gpurun_out/r4f_breakdown.log 2>&1
tail -15 gpurun_out/r4f_breakdown.log
