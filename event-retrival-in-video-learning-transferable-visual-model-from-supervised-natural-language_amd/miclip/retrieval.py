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
    """HBM-resident corpus with a bf16 ranking mirror and the f32 master kept
    for exact re-scoring.

    ``topk`` ranks the bf16 mirror for ``k' = min(REG_K, oversample * k)``
    candidates per query (half the HBM bytes of the f32 pass), gathers the
    union of the candidates' f32 rows (ascending corpus order) and re-ranks
    them with the exact f32 kernel, so scores are bit-identical to
    ``rank_topk(master, ...)``.  The result is certified per query: with the
    mirror's score error bounded by ``delta`` (bf16 rounding of the rows,
    2^-8 relative, on both the dot product and the norm), every row outside the
    k' candidates scores at most ``s_bf16[k'-1] + delta`` exactly, so once the
    exact k-th score exceeds that bound no row outside can enter the top-k.
    Queries that fail the certificate (near-ties across the candidate edge)
    fall back to the exact f32 pass over the master.

    Reference semantics: ``EmbeddingService.search_top_frames`` ranks
    ``get_embeddings`` rows (embedding_service.py:209-210, 314-320); the stored
    ``.npy`` rows stay the f32 master (embedding_service.py:505).
    """

    def __init__(self, master, oversample: int = 4):
        import torch
        if not master.is_cuda:
            raise N.MiClipError("MirroredCorpus lives in HBM: move the master rows to the device first")
        self.master = _corpus(master).float().contiguous()
        self.mirror = self.master.to(torch.bfloat16).contiguous()
        self.oversample = int(oversample)
        self.fallbacks = 0

    def __len__(self):
        return self.master.shape[0]

    def topk(self, queries, k, norm="l2", nan_policy="first"):
        import torch
        q = _queries(queries, self.master.device)
        n = self.master.shape[0]
        kk = min(k, n)
        kc = min(max(REG_K, kk), max(kk, self.oversample * kk), n)
        if kk <= 0:
            return rank_topk(self.master, q, k, norm=norm, nan_policy=nan_policy)
        s1, i1 = rank_topk(self.mirror, q, kc, norm=norm, nan_policy=nan_policy)
        if kc >= n:      # every row is a candidate: the exact pass is the answer
            return rank_topk(self.master, q, k, norm=norm, nan_policy=nan_policy)
        union = torch.unique(i1.flatten())                    # sorted ascending: index ties keep corpus order
        s2, j2 = rank_topk(self.master.index_select(0, union), q, kk, norm=norm, nan_policy=nan_policy)
        i2 = union[j2]
        # certificate: bf16 rows carry a relative error <= 2^-8 per element, so
        # |s_bf16 - s_exact| <= delta = 2^-7 |q| (dot and norm) for "l2";
        # un-normalised scores scale with the row norm, so certify only "l2"
        if norm != "l2":
            self.fallbacks += q.shape[0]
            return rank_topk(self.master, q, k, norm=norm, nan_policy=nan_policy)
        delta = q.norm(dim=1) * 2.0 ** -7
        edge = s1[:, kc - 1]
        ok = (s2[:, kk - 1] > edge + 2 * delta) & torch.isfinite(s2).all(1) & torch.isfinite(s1).all(1)
        if bool(ok.all()):
            return s2, i2
        bad = torch.nonzero(~ok).flatten()
        self.fallbacks += int(bad.numel())
        sf, jf = rank_topk(self.master, q.index_select(0, bad), k, norm=norm, nan_policy=nan_policy)
        s2 = s2.clone()
        i2 = i2.clone()
        s2[bad] = sf
        i2[bad] = jf
        return s2, i2

