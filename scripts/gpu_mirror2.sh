# Mirror: every GPU test, then a rocprofv3 kernel trace of scripts/mirror_micro.py (per-kernel breakdown).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mprof
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mprof -o mirror -- python3 scripts/mirror_micro.py 1 > gpurun_out/mprof/stdout.log 2>&1 || exit $?
grep -v '^{' gpurun_out/mprof/stdout.log | tail -6
find gpurun_out/mprof -name "*kernel_stats.csv" | head -3
