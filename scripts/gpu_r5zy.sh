# r05 zy: the whole GPU suite, smoke, the bench line and a kernel trace on the round-5 final tree (conv1 split from pixels)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zy
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5zy/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r5zy/pytest_gpu.log | tail -30; exit 1; }
tail -2 gpurun_out/r5zy/pytest_gpu.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r5zy/smoke.log 2>&1 || { tail -20 gpurun_out/r5zy/smoke.log; exit 1; }
tail -1 gpurun_out/r5zy/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/r5zy/bench.log 2> gpurun_out/r5zy/bench.err || { tail -20 gpurun_out/r5zy/bench.err; exit 1; }
tail -1 gpurun_out/r5zy/bench.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5zy/prof -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/r5zy/prof.log 2>&1 || exit $?
echo done
