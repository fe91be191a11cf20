# r05 zx: conv1's split operand straight from the pixels (fp32 tower): bit-identity, tower timing, fp32 tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zx
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rk_flow.py -k "conv1 or fp32_tower" \
  > gpurun_out/r5zx/pytest.log 2>&1 || { tail -30 gpurun_out/r5zx/pytest.log; exit 1; }
tail -2 gpurun_out/r5zx/pytest.log


echo done
