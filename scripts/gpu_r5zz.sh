# r05 zz: the secondary configs on the final tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zz
timeout -k 10 300 python bench.py --model ViT-B/32 --frames 125000 --queries 32 --steps 2 --warmup 1 --no-cpu-baseline \
  --no-rank-roofline --no-parity-mode > gpurun_out/r5zz/config3.log 2> gpurun_out/r5zz/config3.err || exit $?
tail -1 gpurun_out/r5zz/config3.log | cut -c1-200
timeout -k 10 500 python bench.py --model ViT-L/14 --frames 100000 --queries 256 --steps 1 --warmup 1 --no-cpu-baseline \
  --no-rank-roofline --no-parity-mode > gpurun_out/r5zz/config2.log 2> gpurun_out/r5zz/config2.err || exit $?
tail -1 gpurun_out/r5zz/config2.log | cut -c1-200
timeout -k 10 500 python bench.py --model ViT-L/14@336px --weights fp8 --frames 125000 --queries 1000 --steps 1 --warmup 1 \
  --no-cpu-baseline --no-rank-roofline > gpurun_out/r5zz/config4.log 2> gpurun_out/r5zz/config4.err || exit $?
tail -1 gpurun_out/r5zz/config4.log | cut -c1-200

echo done
