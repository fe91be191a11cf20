# r05 zh: the whole GPU suite, smoke and the bench line with the parity mode on the 8-phase split-f16 GEMMs; a kernel trace of the bench (rocpd db: step sequence)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zh
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5zh/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r5zh/pytest_gpu.log | tail -30; exit 1; }
tail -2 gpurun_out/r5zh/pytest_gpu.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r5zh/smoke.log 2>&1 || { tail -20 gpurun_out/r5zh/smoke.log; exit 1; }
tail -1 gpurun_out/r5zh/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/r5zh/bench.log 2> gpurun_out/r5zh/bench.err || { tail -20 gpurun_out/r5zh/bench.err; exit 1; }
tail -1 gpurun_out/r5zh/bench.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5zh/prof -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/r5zh/prof.log 2>&1 || exit $?
echo done
