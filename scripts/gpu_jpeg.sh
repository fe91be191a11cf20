# GPU JPEG decode: parity tests, throughput, kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_jpeg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_jpeg.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/jpeg_micro.py 512,2048 > gpurun_out/jpeg_micro.log 2>&1 || exit $?
cat gpurun_out/jpeg_micro.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/jpeg_prof -o j -- python3 scripts/jpeg_micro.py 512 > gpurun_out/jpeg_prof.log 2>&1 || exit $?
grep -h "jpeg" gpurun_out/jpeg_prof/*/j_kernel_stats.csv gpurun_out/jpeg_prof/j_kernel_stats.csv 2>/dev/null | cut -c1-200
