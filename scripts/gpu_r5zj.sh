# r05 zj: the folded tower's last block on the CLS rows only: bit-identity tests, the configs[1] pass check, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zj
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_encode.py tests/test_gpu_bench_config.py tests/test_gpu_rk_flow.py \
  > gpurun_out/r5zj/pytest.log 2>&1 || { tail -30 gpurun_out/r5zj/pytest.log; exit 1; }
tail -2 gpurun_out/r5zj/pytest.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/r5zj/bench.log 2> gpurun_out/r5zj/bench.err || { tail -20 gpurun_out/r5zj/bench.err; exit 1; }
tail -1 gpurun_out/r5zj/bench.log | cut -c1-300
echo done
