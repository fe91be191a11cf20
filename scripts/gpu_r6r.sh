# r06 r: the whole GPU suite, smoke and the bench line on the tree with the batched fp32 attention
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6r
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread \
  > gpurun_out/r6r/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r6r/pytest_gpu.log | tail -30; exit 1; }
tail -2 gpurun_out/r6r/pytest_gpu.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r6r/smoke.log 2>&1 || { tail -20 gpurun_out/r6r/smoke.log; exit 1; }
tail -1 gpurun_out/r6r/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r6r/bench.log 2> gpurun_out/r6r/bench.err || { tail -20 gpurun_out/r6r/bench.err; exit 1; }
tail -1 gpurun_out/r6r/bench.log | cut -c1-400
echo done
