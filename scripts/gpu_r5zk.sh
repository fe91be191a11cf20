# r05 zk: the last block with Q for the CLS rows only (K / V for every row): bit-identity tests, configs[1] check, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zk
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_encode.py tests/test_gpu_bench_config.py tests/test_gpu_rk_flow.py \
  > gpurun_out/r5zk/pytest.log 2>&1 || { tail -30 gpurun_out/r5zk/pytest.log; exit 1; }
tail -2 gpurun_out/r5zk/pytest.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/r5zk/bench.log 2> gpurun_out/r5zk/bench.err || { tail -20 gpurun_out/r5zk/bench.err; exit 1; }
tail -1 gpurun_out/r5zk/bench.log | cut -c1-300
echo done
