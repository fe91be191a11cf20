# r06 k: the whole GPU suite, smoke, the bench line and configs[4] on the current tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6k
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread \
  > gpurun_out/r6k/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r6k/pytest_gpu.log | tail -30; exit 1; }
tail -2 gpurun_out/r6k/pytest_gpu.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r6k/smoke.log 2>&1 || { tail -20 gpurun_out/r6k/smoke.log; exit 1; }
tail -1 gpurun_out/r6k/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r6k/bench.log 2> gpurun_out/r6k/bench.err || { tail -20 gpurun_out/r6k/bench.err; exit 1; }
tail -1 gpurun_out/r6k/bench.log | cut -c1-400
timeout -k 10 500 python bench.py --model ViT-L/14@336px --weights fp8 --frames 125000 --queries 1000 --steps 1 --warmup 1 \
  --no-cpu-baseline --no-rank-roofline > gpurun_out/r6k/config4.log 2> gpurun_out/r6k/config4.err || { tail -20 gpurun_out/r6k/config4.err; exit 1; }
tail -1 gpurun_out/r6k/config4.log | cut -c1-300
echo done
