# r05 zl: the MX-fp8 tower's last block on the CLS rows (bit-identity), then the secondary configs on the tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zl
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_mx.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r5zl/pytest.log 2>&1 || { tail -30 gpurun_out/r5zl/pytest.log; exit 1; }
tail -2 gpurun_out/r5zl/pytest.log
timeout -k 10 300 python bench.py --model ViT-B/32 --frames 125000 --queries 32 --steps 2 --warmup 1 --no-cpu-baseline \
  --no-rank-roofline --no-parity-mode > gpurun_out/r5zl/config3.log 2> gpurun_out/r5zl/config3.err || exit $?
tail -1 gpurun_out/r5zl/config3.log | cut -c1-200
timeout -k 10 500 python bench.py --model ViT-L/14 --frames 100000 --queries 256 --steps 1 --warmup 1 --no-cpu-baseline \
  --no-rank-roofline --no-parity-mode > gpurun_out/r5zl/config2.log 2> gpurun_out/r5zl/config2.err || exit $?
tail -1 gpurun_out/r5zl/config2.log | cut -c1-200
timeout -k 10 500 python bench.py --model ViT-L/14@336px --weights fp8 --frames 125000 --queries 1000 --steps 1 --warmup 1 \
  --no-cpu-baseline --no-rank-roofline > gpurun_out/r5zl/config4.log 2> gpurun_out/r5zl/config4.err || exit $?
tail -1 gpurun_out/r5zl/config4.log | cut -c1-200

timeout -k 10 200 python -u scripts/text_micro.py 32 5 > gpurun_out/r5zl/text_micro.log 2>&1 || { cat gpurun_out/r5zl/text_micro.log; exit 1; }
grep -v "amdgpu.ids\|Warning\|api.load" gpurun_out/r5zl/text_micro.log
echo done
