# Round 3: JPEG v2 (queue reader in the chunk passes, workgroup unstuff, 4-px colour): tests, breakdown, kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_service.py tests/test_gpu_flows.py -q --timeout 300 --timeout-method thread > gpurun_out/r3d_jpeg_tests.log 2>&1
rc=$?; echo "jpeg tests rc=$rc"; tail -5 gpurun_out/r3d_jpeg_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python scripts/jpeg_breakdown.py 8192 > gpurun_out/r3d_breakdown.log 2>&1 || exit $?
cat gpurun_out/r3d_breakdown.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3d_jprof -o jp -- python3 scripts/jpeg_micro.py 8192 > gpurun_out/r3d_jprof.log 2>&1 || exit $?
tail -2 gpurun_out/r3d_jprof.log
cut -d, -f1-4 gpurun_out/r3d_jprof/jp_kernel_stats.csv | sed 's/miclip::(anonymous namespace):://; s/(.*)"/"/' | head -16
