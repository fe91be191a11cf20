# r05 b: the fp32 tower on split-f16 GEMMs + the exact-f32 MFMA attention: the new op tests,
# then the whole GPU suite, then the default bench line (parity_mode inside) and a kernel trace
# of the parity mode
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5b
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread \
  -k "split2h or attention_f32" > gpurun_out/r5b/pytest_ops.log 2>&1 || { tail -40 gpurun_out/r5b/pytest_ops.log; exit 1; }
tail -2 gpurun_out/r5b/pytest_ops.log
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5b/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r5b/pytest_gpu.log | tail -30; exit 1; }
tail -2 gpurun_out/r5b/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/r5b/bench.log 2> gpurun_out/r5b/bench.err || { tail -20 gpurun_out/r5b/bench.err; exit 1; }
tail -1 gpurun_out/r5b/bench.log | cut -c1-600
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5b/prof_fp32 -o bench -- \
  python3 bench.py --weights fp32 --steps 2 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-kernel-timing \
  > gpurun_out/r5b/prof_fp32.log 2>&1 || exit $?
echo done
