"""The product rank route at BASELINE config scale against the float64 oracle
(the certified pass, the mirror and the shard merge were only
compared with the A/B exact pass above 50k rows).

Reference semantics: ``np.dot(E_normalised, t.T)`` + ``np.argsort(s)[::-1][:k]``
(Backend/services/embedding_service.py:209-210, 314-320), in the deterministic
order rule (score desc, index asc).  The oracle here is the float64 scores of
the same rows (chunked, so 1M x 768 fits), top-k by (score desc, index asc):
the kernel's indices must be those, except where two float64 scores are closer
than the f32 tolerance (2e-6, rank_ref.assert_topk_equivalent's), and its
scores within 8e-6 of float64.

Shapes:
  1M x 512, Q = 32, k = 10, f32 and bf16 rows  the certified bf16-MFMA pass (default >= 262144 rows)
  100k x 768, Q = 256, k = 10                  configs[2]'s rank shape
  8 shards x 125k x 512, Q = 32, merged         configs[3] (one process, index_base + mi_rank_merge)
  1M x 768, Q = 1000, k = 10, MirroredCorpus    configs[4]'s rank shape
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 2e-6


def _rows(seed, n, d, near=None):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((n, d), dtype=np.float32)
    c *= rng.uniform(0.5, 2.0, (n, 1)).astype(np.float32)       # un-normalised rows of varied norm
    return c


def _queries(seed, q, d, corpus=None, n_near=0):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((q, d))
    if corpus is not None and n_near:
        pick = rng.integers(0, corpus.shape[0], n_near)
        x[:n_near] = corpus[pick] / np.linalg.norm(corpus[pick], axis=1, keepdims=True) * 6 + x[:n_near] * 0.2
    return (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)


def _oracle_topk(corpus, q, k, chunk=65536, extra=8):
    """float64 top-(k+extra) candidates per query of <q, c/|c|> over all rows,
    ordered (score desc, index asc)."""
    Q = q.shape[0]
    q64 = q.astype(np.float64)
    best_s = np.full((Q, 0), -np.inf)
    best_i = np.zeros((Q, 0), np.int64)
    m = k + extra
    for a in range(0, corpus.shape[0], chunk):
        c = corpus[a:a + chunk].astype(np.float64)
        c /= np.linalg.norm(c, axis=1, keepdims=True)
        s = q64 @ c.T                                            # [Q, chunk]
        take = min(m, s.shape[1])
        part = np.argpartition(-s, take - 1, axis=1)[:, :take]
        best_s = np.concatenate([best_s, np.take_along_axis(s, part, 1)], 1)
        best_i = np.concatenate([best_i, part + a], 1)
        if best_s.shape[1] > m:
            keep = np.argpartition(-best_s, m - 1, axis=1)[:, :m]
            best_s = np.take_along_axis(best_s, keep, 1)
            best_i = np.take_along_axis(best_i, keep, 1)
    order = np.lexsort((best_i, -best_s), axis=1)
    return np.take_along_axis(best_s, order, 1), np.take_along_axis(best_i, order, 1)


def _exact_scores(corpus, q, idx):
    """float64 <q, c/|c|> of the rows idx [Q, k]."""
    c = corpus[idx].astype(np.float64)                           # [Q, k, D]
    c /= np.linalg.norm(c, axis=2, keepdims=True)
    return np.einsum("qkd,qd->qk", c, q.astype(np.float64))


def _check(corpus, q, k, got_s, got_i, ref_s, ref_i):
    got_s, got_i = np.asarray(got_s), np.asarray(got_i)
    assert got_i.shape == (q.shape[0], k)
    exp = _exact_scores(corpus, q, got_i)
    np.testing.assert_allclose(got_s, exp, rtol=0, atol=4 * TOL)
    swaps = 0
    for r in range(q.shape[0]):
        assert len(set(got_i[r].tolist())) == k, f"query {r}: duplicate indices"
        for p in range(k):
            if got_i[r, p] != ref_i[r, p]:
                assert abs(exp[r, p] - ref_s[r, p]) < TOL, \
                    f"query {r} pos {p}: got {got_i[r, p]} ({exp[r, p]}), oracle {ref_i[r, p]} ({ref_s[r, p]})"
                swaps += 1
    return swaps


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_certified_pass_1m_vs_oracle(gpu, dt):
    """1M x 512, Q = 32, k = 10 (the certified bf16-MFMA pass, the product default for
    f32 / bf16 rows of >= 262144 rows) against float64."""
    import torch
    from miclip import retrieval
    c = _rows(1, 1_000_000, 512)
    q = _queries(2, 32, 512, c, n_near=8)
    t = torch.from_numpy(c).to(gpu)
    if dt == "bf16":
        t = t.bfloat16()
        c = t.float().cpu().numpy()                               # the oracle scores the bf16 values
    s, i = retrieval.rank_topk(t, torch.from_numpy(q).to(gpu), 10)
    ref_s, ref_i = _oracle_topk(c, q, 10)
    assert _check(c, q, 10, s.cpu().numpy(), i.cpu().numpy(), ref_s, ref_i) <= 2


def test_configs2_rank_shape_vs_oracle(gpu):
    """configs[2]'s rank shape: 100k x 768 corpus, Q = 256 queries, k = 10."""
    import torch
    from miclip import retrieval
    c = _rows(3, 100_000, 768)
    q = _queries(4, 256, 768, c, n_near=64)
    s, i = retrieval.rank_topk(torch.from_numpy(c).to(gpu), torch.from_numpy(q).to(gpu), 10)
    ref_s, ref_i = _oracle_topk(c, q, 10)
    assert _check(c, q, 10, s.cpu().numpy(), i.cpu().numpy(), ref_s, ref_i) <= 4


def test_configs3_sharded_merge_vs_oracle(gpu):
    """configs[3]: 1M rows as 8 contiguous 125k shards (index_base = r * 125k), each
    ranked on its own, the [Q, 8k] candidates merged by mi_rank_merge (the RCCL
    all-gather's payload, miclip/distributed.py) -- against float64 over all 1M."""
    import torch
    from miclip import retrieval
    c = _rows(5, 1_000_000, 512)
    q = _queries(6, 32, 512, c, n_near=8)
    qt = torch.from_numpy(q).to(gpu)
    P, n = 8, 125_000
    cs, ci = [], []
    for r in range(P):
        s, i = retrieval.rank_topk(torch.from_numpy(c[r * n:(r + 1) * n]).to(gpu), qt, 10, index_base=r * n)
        cs.append(s)
        ci.append(i)
    s, i = retrieval.merge_topk(torch.cat(cs, 1), torch.cat(ci, 1), 10)
    ref_s, ref_i = _oracle_topk(c, q, 10)
    assert _check(c, q, 10, s.cpu().numpy(), i.cpu().numpy(), ref_s, ref_i) <= 2


def test_configs4_mirror_q1000_vs_oracle(gpu):
    """configs[4]'s rank shape through the product route for large corpora
    (retrieval.MirroredCorpus: fp16 mirror pass, certified exact re-score, the
    uncertified queries through the exact pass): 1M x 768, Q = 1000, k = 10."""
    import torch
    from miclip import retrieval
    c = _rows(7, 1_000_000, 768)
    q = _queries(8, 1000, 768, c, n_near=200)
    mc = retrieval.MirroredCorpus(torch.from_numpy(c).to(gpu))
    s, i = mc.topk(torch.from_numpy(q).to(gpu), 10)
    assert mc.certified + mc.fallbacks == 1000 and mc.certified >= 900
    ref_s, ref_i = _oracle_topk(c, q, 10)
    assert _check(c, q, 10, s.cpu().numpy(), i.cpu().numpy(), ref_s, ref_i) <= 8
