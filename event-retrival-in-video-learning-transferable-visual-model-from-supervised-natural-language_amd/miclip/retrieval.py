"""Device-side ranking: the fused normalise + cosine + top-k kernel and the
R@K helpers, behind torch tensors.

Reference call sites this replaces:
  ``np.dot(embeddings, text_features.T)`` + ``np.argsort(s)[::-1][:top_k]``
      Backend/services/embedding_service.py:314-320 (text) and :365-372 (image query)
  ``image_features @ text_features.T`` + per-query ``np.argsort(-s)`` rank of GT
      Backend/content/Test_compare_model/compare_models.py:999-1016, 1045-1062

Order rule (documented in include/miclip.h): score descending, then index
ascending; NaN (a zero-norm row divided by its norm) first for the
``search_top_frames`` semantics (``argsort(s)[::-1]``), last for the
``compare_models`` semantics (``argsort(-s)``).
"""
from __future__ import annotations

import threading

from . import _native as N

_NORMS = {"l2": N.MI_NORM_L2, "l2_guard": N.MI_NORM_L2_GUARD, "none": N.MI_NORM_NONE}
_NANS = {"first": N.MI_NAN_FIRST, "last": N.MI_NAN_LAST}
REG_K = 64          # fused single-pass top-k (register lists) up to this k
MAX_K = 1 << 24     # above REG_K: exact scores + radix select + sort (rank.hip)
MAX_D = 1024

_ws_lock = threading.Lock()
_ws = {}


def _workspace(device, nbytes):
    """Scratch for mi_rank_topk, one buffer per (device, stream): kernels of
    two threads on different streams never share it (same-stream callers are
    ordered by the stream)."""
    import torch
    key = (device, N.stream_ptr(device))
    with _ws_lock:
        buf = _ws.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
            _ws[key] = buf
        return buf


def _corpus(corpus):
    import torch
    if corpus.dim() != 2:
        raise N.MiClipError("corpus must be [N, D]")
    if corpus.dtype not in (torch.float32, torch.bfloat16, torch.float16):
        corpus = corpus.float()
    return corpus.contiguous()


def _queries(queries, device):
    import torch
    q = queries if queries.dim() == 2 else queries.reshape(1, -1)
    return q.to(device=device, dtype=torch.float32).contiguous()


def rank_topk(corpus, queries, k, index_base=0, norm="l2", nan_policy="first"):
    """Top-k rows of ``corpus`` [N,D] (device) for each query [Q,D].

    Returns (scores f32 [Q, min(k,N)], index int64 [Q, min(k,N)]) on the device.
    """
    import torch
    if not corpus.is_cuda:
        raise N.MiClipError("rank_topk runs on the GPU: move the corpus to the device first")
    c = _corpus(corpus)
    q = _queries(queries, c.device)
    if q.shape[1] != c.shape[1]:
        raise N.MiClipError(f"dimension mismatch: corpus D={c.shape[1]}, queries D={q.shape[1]}")
    Nrows, D = c.shape
    Q = q.shape[0]
    if not 1 <= k <= MAX_K:
        raise N.MiClipError(f"k must be in [1, {MAX_K}]")
    if not (32 <= D <= MAX_D and D % 32 == 0):
        raise N.MiClipError(f"D must be a multiple of 32 in [32, {MAX_D}], got {D}")
    out_s = torch.empty((Q, k), dtype=torch.float32, device=c.device)
    out_i = torch.empty((Q, k), dtype=torch.int64, device=c.device)
    L = N.lib()
    nbytes = L.mi_rank_workspace_bytes(Nrows, Q, k)
    with torch.cuda.device(c.device):
        ws = _workspace(c.device, nbytes)
        N.check(L.mi_rank_topk(c.data_ptr(), Nrows, D, N.dtype_code(c.dtype), q.data_ptr(), Q, k, int(index_base),
                               _NORMS[norm], _NANS[nan_policy], out_s.data_ptr(), out_i.data_ptr(), ws.data_ptr(),
                               ws.numel(), N.stream_ptr(c.device)), "mi_rank_topk")
    kk = min(k, Nrows)
    return out_s[:, :kk], out_i[:, :kk]


def normalize_rows_f16(rows, out=None):
    """``embeddings / np.linalg.norm(embeddings, axis=-1, keepdims=True)`` for a
    float16 corpus, bit for bit as NumPy evaluates it in float16
    (Backend/services/embedding_service.py:209-210 on the reference's fp16
    ``.npy`` files; ``mi_normalize_rows_f16``, csrc/corpus.hip).  ``rows``: device
    fp16 [N, D]; returns the normalised fp16 rows (``out`` may be ``rows``)."""
    import torch
    if not rows.is_cuda or rows.dtype != torch.float16 or rows.dim() != 2:
        raise N.MiClipError("normalize_rows_f16 takes device float16 [N, D] rows")
    r = rows.contiguous()
    o = torch.empty_like(r) if out is None else out
    if o.shape != r.shape or o.dtype != torch.float16 or not o.is_contiguous():
        raise N.MiClipError("normalize_rows_f16: out must be contiguous float16 of the rows' shape")
    with torch.cuda.device(r.device):
        N.check(N.lib().mi_normalize_rows_f16(r.data_ptr(), r.shape[0], r.shape[1], o.data_ptr(),
                                              N.stream_ptr(r.device)), "mi_normalize_rows_f16")
    return o


def merge_topk(cand_scores, cand_index, k, nan_policy="first"):
    """Merge [Q, C] candidate lists (index -1 = empty) into the top-k (device)."""
    import torch
    s = cand_scores.to(torch.float32).contiguous()
    i = cand_index.to(torch.int64).contiguous()
    Q, C = s.shape
    out_s = torch.empty((Q, k), dtype=torch.float32, device=s.device)
    out_i = torch.empty((Q, k), dtype=torch.int64, device=s.device)
    with torch.cuda.device(s.device):
        N.check(N.lib().mi_rank_merge(s.data_ptr(), i.data_ptr(), Q, C, k, _NANS[nan_policy], out_s.data_ptr(),
                                      out_i.data_ptr(), N.stream_ptr(s.device)), "mi_rank_merge")
    return out_s, out_i


def score_matrix(corpus, queries, norm="none"):
    """[Q, N] f32 scores <q, c/|c|> with fp32-exact products (device)."""
    import torch
    c = _corpus(corpus)
    q = _queries(queries, c.device)
    out = torch.empty((q.shape[0], c.shape[0]), dtype=torch.float32, device=c.device)
    with torch.cuda.device(c.device):
        N.check(N.lib().mi_score_matrix(c.data_ptr(), c.shape[0], c.shape[1], N.dtype_code(c.dtype), q.data_ptr(),
                                        q.shape[0], _NORMS[norm], out.data_ptr(), N.stream_ptr(c.device)),
                "mi_score_matrix")
    return out


def rank_of_targets(scores, pair_query, pair_target):
    """1-based rank of scores[q, g] in argsort(-scores[q]) for each (q, g) pair."""
    import torch
    s = scores.to(torch.float32).contiguous()
    pq = torch.as_tensor(pair_query, dtype=torch.int64).to(s.device).contiguous()
    pt = torch.as_tensor(pair_target, dtype=torch.int64).to(s.device).contiguous()
    out = torch.empty(pq.shape[0], dtype=torch.int64, device=s.device)
    with torch.cuda.device(s.device):
        N.check(N.lib().mi_rank_of_targets(s.data_ptr(), s.shape[0], s.shape[1], pq.data_ptr(), pt.data_ptr(),
                                           pq.shape[0], out.data_ptr(), N.stream_ptr(s.device)),
                "mi_rank_of_targets")
    return out


class MirroredCorpus:
    """HBM-resident corpus with an fp16 ranking mirror and the master kept for
    exact re-scoring (csrc/rank_mirror.hip).

    The mirror holds every row as an fp16 unit vector (``mi_mirror_build``,
    the exact path's reciprocal norm), so ``topk`` streams half the f32 bytes
    on the fp16 MFMA for the top 16 mirror candidates per query, re-scores
    them against the master with the exact path's arithmetic, and certifies
    the result per query: with the mirror's score error bounded by delta
    (rank_mirror.hip), every row outside the candidates scores at most
    ``s_mirror[15] + delta``, so once the exact k-th score exceeds that bound
    the answer is bit-identical to ``rank_topk(master, ...)``.  Queries that
    fail the certificate (near-ties across the candidate edge, NaN rows) and
    requests the mirror does not cover (k > MAX_K, norm other than "l2",
    D not in {512, 768}) take the exact pass; ``fallbacks`` counts them.
    MAX_K = 12 < 16: the certificate needs a score gap between the k-th
    exact and the 16th mirror candidate, which k = 16 never has.

    Reference semantics: ``EmbeddingService.search_top_frames`` ranks
    ``get_embeddings`` rows (embedding_service.py:209-210, 314-320); the stored
    ``.npy`` rows stay the master (embedding_service.py:505).
    """

    MAX_K = 12

    def __init__(self, master):
        import torch
        if not master.is_cuda:
            raise N.MiClipError("MirroredCorpus lives in HBM: move the master rows to the device first")
        self.master = _corpus(master)
        n, d = self.master.shape
        self.mirror = None
        self.fallbacks = 0
        self.certified = 0
        if n > 0 and d in (512, 768):
            self.mirror = torch.empty((n, d), dtype=torch.float16, device=self.master.device)
            with torch.cuda.device(self.master.device):
                N.check(N.lib().mi_mirror_build(self.master.data_ptr(), n, d, N.dtype_code(self.master.dtype),
                                                self.mirror.data_ptr(), N.stream_ptr(self.master.device)),
                        "mi_mirror_build")

    def __len__(self):
        return self.master.shape[0]

    def topk(self, queries, k, norm="l2", nan_policy="first", index_base=0):
        import torch
        q = _queries(queries, self.master.device)
        n, d = self.master.shape
        Q = q.shape[0]
        if q.shape[1] != d:
            raise N.MiClipError(f"dimension mismatch: corpus D={d}, queries D={q.shape[1]}")
        if self.mirror is None or norm != "l2" or not 1 <= k <= self.MAX_K or Q == 0:
            self.fallbacks += Q
            return rank_topk(self.master, q, k, index_base=index_base, norm=norm, nan_policy=nan_policy)
        dev = self.master.device
        out_s = torch.empty((Q, k), dtype=torch.float32, device=dev)
        out_i = torch.empty((Q, k), dtype=torch.int64, device=dev)
        cert = torch.empty(Q, dtype=torch.int32, device=dev)
        L = N.lib()
        with torch.cuda.device(dev):
            ws = _workspace(dev, L.mi_rank_mirror_workspace_bytes(n, Q))
            N.check(L.mi_rank_mirror(self.mirror.data_ptr(), self.master.data_ptr(), n, d,
                                     N.dtype_code(self.master.dtype), q.data_ptr(), Q, k, int(index_base),
                                     _NANS[nan_policy], out_s.data_ptr(), out_i.data_ptr(), cert.data_ptr(),
                                     ws.data_ptr(), ws.numel(), N.stream_ptr(dev)), "mi_rank_mirror")
        bad = torch.nonzero(cert == 0).flatten()
        nb = int(bad.numel())
        self.fallbacks += nb
        self.certified += Q - nb
        if nb:
            sf, jf = rank_topk(self.master, q.index_select(0, bad), k, index_base=index_base, norm=norm,
                               nan_policy=nan_policy)
            out_s[bad, :sf.shape[1]] = sf
            out_i[bad, :jf.shape[1]] = jf
        kk = min(k, n)
        return out_s[:, :kk], out_i[:, :kk]
