# r05 zu: the last block's attention on the CLS queries' tile only (bf16 S <= 64, fp32 MFMA): bit-identity tests, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zu
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rk_flow.py \
  tests/test_gpu_encode.py tests/test_gpu_bench_config.py tests/test_gpu_ops.py -k "cls_rows or fp32 or rk_flow or attention or bench_config or lnfold" \
  > gpurun_out/r5zu/pytest.log 2>&1 || { tail -30 gpurun_out/r5zu/pytest.log; exit 1; }
tail -2 gpurun_out/r5zu/pytest.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/r5zu/bench.log 2> gpurun_out/r5zu/bench.err || { tail -20 gpurun_out/r5zu/bench.err; exit 1; }
tail -1 gpurun_out/r5zu/bench.log | cut -c1-200
echo done
