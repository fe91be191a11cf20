"""Sharded retrieval on the GPU: per-shard fused top-k with
global ``index_base`` + the HIP merge of the gathered [Q, P*k] candidates must
equal the single-device top-k bit for bit (same exact-f32 scores, same
(score desc, index asc) rule), and the RCCL process group the bench opens
(``init_process_group("nccl", device_id=...)``) must come up and all-gather on
this box.  The collective logic at world_size 2/3 is covered on CPU with gloo
(tests/test_distributed.py); a one-GPU box cannot host two RCCL ranks."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,n,q,k", [(2, 10007, 32, 10), (3, 4099, 7, 5), (8, 20000, 32, 10)])
def test_shard_merge_matches_global(gpu, world, n, q, k):
    import torch
    from miclip import distributed, retrieval, weights
    from oracle import rank_ref
    corpus = torch.from_numpy(weights.normal(11, "shard-corpus", (n, 512))).to(gpu)
    corpus[n // 3] = corpus[n // 5]                    # an exact tie across shards
    queries = torch.from_numpy(weights.synthetic_corpus(q, 512, seed=12)).to(gpu)
    ss, ii = [], []
    for r in range(world):
        s0, e0 = distributed.shard_range(n, world, r)
        s, i = retrieval.rank_topk(corpus[s0:e0], queries, k, index_base=s0)
        s, i = distributed._pad(s, i, k)
        ss.append(s)
        ii.append(i)
    ms, mi = retrieval.merge_topk(torch.cat(ss, 1), torch.cat(ii, 1), k)
    gs, gi = retrieval.rank_topk(corpus, queries, k)
    assert torch.equal(mi, gi) and torch.equal(ms, gs)
    S = rank_ref.scores_ref(corpus.cpu().numpy(), queries.cpu().numpy())
    for r in range(q):
        rank_ref.assert_topk_equivalent(ms[r].cpu().numpy(), mi[r].cpu().numpy(), S[r], k)


_RCCL_CHILD = r"""
import os, sys, torch, torch.distributed as dist
sys.path[:0] = [os.environ["MICLIP_PKG"], os.environ["MICLIP_ROOT"]]
from miclip import distributed, retrieval, weights
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
corpus = torch.from_numpy(weights.normal(13, "rccl-corpus", (5000, 512))).to(dev)
queries = torch.from_numpy(weights.synthetic_corpus(16, 512, seed=14)).to(dev)
s, i = distributed.sharded_topk(corpus, queries, 10, 0)
gs, gi = retrieval.rank_topk(corpus, queries, 10)
assert torch.equal(s, gs) and torch.equal(i, gi)
out = [torch.empty_like(s)]
dist.all_gather(out, s)
oi = [torch.empty_like(i)]
dist.all_gather(oi, i)
torch.cuda.synchronize(dev)
assert torch.equal(out[0], s) and torch.equal(oi[0], i)
t = torch.tensor([1.5], device=dev, dtype=torch.float64)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
assert t.item() == 1.5
dist.barrier()
dist.destroy_process_group()
print("rccl ok")
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_group_single_rank(gpu):
    """The bench's RCCL init + all_gather / all_reduce(MAX) / barrier on GPU
    tensors, in a child process (its own HIP context and process group)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), MICLIP_PKG=PKG,
               MICLIP_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", _RCCL_CHILD], env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "rccl ok" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
