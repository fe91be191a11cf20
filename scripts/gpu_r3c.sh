# Round 3: chunked JPEG entropy decode — GPU JPEG tests, then the JPEG micro + an entropy-kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py -v --timeout 300 --timeout-method thread > gpurun_out/r3c_jpeg_tests.log 2>&1
rc=$?; echo "jpeg tests rc=$rc"; grep -E "PASS|FAIL|ERROR|Error|error" gpurun_out/r3c_jpeg_tests.log | tail -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python scripts/jpeg_micro.py 2048,8192 > gpurun_out/r3c_jpeg_micro.log 2>&1 || exit $?
tail -5 gpurun_out/r3c_jpeg_micro.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3c_jprof -o jp -- python3 scripts/jpeg_micro.py 8192 > gpurun_out/r3c_jprof.log 2>&1 || exit $?
head -20 gpurun_out/r3c_jprof/jp_kernel_stats.csv
