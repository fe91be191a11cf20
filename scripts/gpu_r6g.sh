# r06 g: the secondary configs on the round-6 tree (configs[3] one 125k-frame B/32 shard, configs[2]
# ViT-L/14 100k x 256, configs[4] one 125k-frame L/14@336 MX-fp8 shard x 1000 queries)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6g
timeout -k 10 300 python bench.py --model ViT-B/32 --frames 125000 --queries 32 --steps 2 --warmup 1 --no-cpu-baseline \
  --no-rank-roofline --no-parity-mode > gpurun_out/r6g/config3.log 2> gpurun_out/r6g/config3.err || { tail -5 gpurun_out/r6g/config3.err; exit 1; }
tail -1 gpurun_out/r6g/config3.log | cut -c1-200
timeout -k 10 500 python bench.py --model ViT-L/14 --frames 100000 --queries 256 --steps 1 --warmup 1 --no-cpu-baseline \
  --no-rank-roofline --no-parity-mode > gpurun_out/r6g/config2.log 2> gpurun_out/r6g/config2.err || { tail -5 gpurun_out/r6g/config2.err; exit 1; }
tail -1 gpurun_out/r6g/config2.log | cut -c1-200
timeout -k 10 500 python bench.py --model ViT-L/14@336px --weights fp8 --frames 125000 --queries 1000 --steps 1 --warmup 1 \
  --no-cpu-baseline --no-rank-roofline > gpurun_out/r6g/config4.log 2> gpurun_out/r6g/config4.err || { tail -5 gpurun_out/r6g/config4.err; exit 1; }
tail -1 gpurun_out/r6g/config4.log | cut -c1-200
echo done
