"""Probe: can two RCCL ranks share one GPU (the 1-GPU box)?  Each rank binds cuda:0 and
all-gathers a small tensor over backend "nccl" (RCCL).
usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
           scripts/probes/rccl_two_ranks_one_gpu.py"""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((4,), float(rank), device="cuda:0")
out = [torch.empty_like(x) for _ in range(world)]
dist.all_gather(out, x)
torch.cuda.synchronize()
print(f"rank {rank}: all_gather {[o.tolist() for o in out]}", flush=True)
dist.destroy_process_group()
