# GPU check + rank A/B: every GPU test, smoke, rank_micro (interleaved vs contiguous tiles), bench line.
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python scripts/rank_micro.py 3 > gpurun_out/rank_micro.log 2>&1 || exit $?
grep -v '^{' gpurun_out/rank_micro.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > gpurun_out/bench.log 2>&1 || exit $?
tail -c 3000 gpurun_out/bench.log
