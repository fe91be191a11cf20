# r06 a: the new config-scale tests first (configs[2] / configs[4] bench passes, S = 197 CLS-row
# block), then the whole GPU suite, smoke and the bench line on the counted-wait tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6a
timeout -k 10 600 python -u -m pytest tests/test_gpu_config_scale.py "tests/test_gpu_rank.py::test_split_merge_static_frames_no_cliff" -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r6a/pytest_config_scale.log 2>&1 || { grep -E "FAILED|Error|passed|failed|assert" gpurun_out/r6a/pytest_config_scale.log | tail -30; exit 1; }
grep -E "chunk|passed|failed" gpurun_out/r6a/pytest_config_scale.log | tail -6
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_config_scale.py \
  > gpurun_out/r6a/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r6a/pytest_gpu.log | tail -30; exit 1; }
tail -2 gpurun_out/r6a/pytest_gpu.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r6a/smoke.log 2>&1 || { tail -20 gpurun_out/r6a/smoke.log; exit 1; }
tail -1 gpurun_out/r6a/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/r6a/bench.log 2> gpurun_out/r6a/bench.err || { tail -20 gpurun_out/r6a/bench.err; exit 1; }
tail -1 gpurun_out/r6a/bench.log | cut -c1-600
echo done
