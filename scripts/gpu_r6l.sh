# r06 l: the multi-rank bench step rehearsed on the one-GPU box: 2 ranks sharing the GPU over gloo
# (RCCL refuses two ranks on one device; the driver's 8-GPU run takes nccl), real kernels, the
# all-gather of per-shard top-k, max-over-ranks timing and the JSON line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6l
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --dist-backend gloo --frames 4000 --steps 2 --warmup 1 --no-cpu-baseline --no-rank-roofline \
  > gpurun_out/r6l/bench2.log 2> gpurun_out/r6l/bench2.err || { tail -30 gpurun_out/r6l/bench2.err; exit 1; }
tail -1 gpurun_out/r6l/bench2.log | cut -c1-700
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 3 --dist-backend gloo --global-frames 9001 --steps 2 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-kernel-timing \
  > gpurun_out/r6l/bench3.log 2> gpurun_out/r6l/bench3.err || { tail -30 gpurun_out/r6l/bench3.err; exit 1; }
tail -1 gpurun_out/r6l/bench3.log | cut -c1-500
echo done
