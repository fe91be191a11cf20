"""CPU, world_size 2 (gloo): the sharded retrieval collective path
(miclip.distributed.sharded_topk) with the oracle as the per-shard top-k and
the merge, checked against the single-process global answer."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q, k, nan_policy, ret):
    import sys
    import torch
    import torch.distributed as dist
    from conftest import PKG, ROOT
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    from miclip import distributed, weights
    from oracle import rank_ref

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    corpus = weights.normal(5, "dist-corpus", (n, 64))
    corpus[7] = 0.0                                   # one NaN row
    queries = weights.synthetic_corpus(q, 64, seed=6)
    s0, e0 = distributed.shard_range(n, world, rank)

    def local(c, qq, kk, index_base, norm, nan_policy):
        s, i = rank_ref.topk_ref(c.numpy(), qq.numpy(), kk, index_base=index_base, nan_policy=nan_policy)
        return torch.from_numpy(s.astype(np.float32)), torch.from_numpy(i)

    def merge(cs, ci, kk, nan_policy):
        s, i = rank_ref.merge_ref(cs.numpy(), ci.numpy(), kk, nan_policy=nan_policy)
        return torch.from_numpy(s.astype(np.float32)), torch.from_numpy(i)

    s, i = distributed.sharded_topk(torch.from_numpy(corpus[s0:e0]), torch.from_numpy(queries), k, s0,
                                    nan_policy=nan_policy, local_topk=local, merge=merge)
    ret[rank] = (s.numpy(), i.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,k,pol", [(2, 1000, 10, "first"), (2, 15, 10, "last"), (3, 500, 64, "first")])
def test_sharded_topk_gloo(world, n, k, pol):
    import multiprocessing as mp
    import torch.multiprocessing as tmp
    from miclip import weights
    from oracle import rank_ref

    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, 4, k, pol, ret)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    del tmp
    corpus = weights.normal(5, "dist-corpus", (n, 64))
    corpus[7] = 0.0
    queries = weights.synthetic_corpus(4, 64, seed=6)
    gs, gi = rank_ref.topk_ref(corpus, queries, k, nan_policy=pol)
    for r in range(world):
        s, i = ret[r]
        kk = min(k, n)
        assert np.array_equal(i[:, :kk], gi)
        assert np.allclose(s[:, :kk], gs, equal_nan=True, atol=1e-6)
        if kk < k:
            assert (i[:, kk:] == -1).all()
