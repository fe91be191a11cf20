# r04: LayerNorm-folded vision tower — encoder parity tests, a bench line and a kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4b
timeout -k 10 900 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_flows.py tests/test_gpu_rk_flow.py \
  tests/test_gpu_ops.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/r4b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r4b_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-parity-mode > gpurun_out/r4b_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r4b_bench.log | cut -c1-600
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4b -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/prof4b/stdout.log 2>&1 || exit $?
find gpurun_out/prof4b -name "*kernel_stats.csv" | head -2
