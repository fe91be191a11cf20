"""ORACLE (test infrastructure only) — NumPy restatement of the reference's
ranking and R@K evaluation.

* ``search_top_frames_ref``: Backend/services/embedding_service.py:209-210
  (``E / ||E||`` at load) and :314-336 (``np.dot(E, t.T).flatten()``,
  ``np.argsort(s)[::-1][:top_k]``, stable re-sort of (frame, sim) pairs by sim
  descending) — the literal reference algorithm, used to pin the fixtures.
* ``topk_ref``: the deterministic order the HIP kernel implements
  (score desc, index asc; NaN first/last), computed in float64 from the same
  normalised rows; equals ``search_top_frames_ref`` whenever there are no exact
  ties (asserted by the fixtures).
* ``retrieval_metrics_ref``: compare_models.py:994-1090 (t2i / i2t ranks via
  ``np.argsort(-s)``, R@1/5/10, MRR, median/mean rank, mean, rsum).
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np


def normalize_rows(E):
    """embedding_service.py:210 — zero rows become NaN (0/0)."""
    with np.errstate(invalid="ignore", divide="ignore"):
        return E / np.linalg.norm(E, axis=-1, keepdims=True)


def pairwise_plan(D):
    """NumPy's pairwise summation tree for a length-D reduction
    (numpy/_core/src/umath/loops_utils.h.src ``pairwise_sum``): leaves of
    <= 128 elements as (start, length) and a postfix program (0 = next leaf,
    1 = add the top two).  csrc/corpus.hip's host plan, restated."""
    leaves, ops = [], []

    def rec(off, n):
        if n <= 128:
            leaves.append((off, n))
            ops.append(0)
            return
        n2 = n // 2
        n2 -= n2 % 8
        rec(off, n2)
        rec(off + n2, n - n2)
        ops.append(1)
    rec(0, D)
    return leaves, ops


def normalize_rows_f16(E16):
    """``E / np.linalg.norm(E, axis=-1, keepdims=True)`` for a float16 array,
    restated step by step as NumPy evaluates it (embedding_service.py:209-210
    on the reference's float16 files; the arithmetic csrc/corpus.hip replays):
    f16 squares, pairwise f32 sum of all D squares from the identity 0 (leaf:
    n < 8 sequential, else 8 strided accumulators ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
    + sequential tail), f16 round, f32 sqrt -> f16, f16(f32 x / f32 norm).
    Pinned against NumPy itself by tests/test_oracle.py."""
    f32 = np.float32
    X = np.asarray(E16, dtype=np.float16)
    R, D = X.shape
    sq = (X * X).astype(f32)                      # HALF_multiply: f16 squares
    leaves, ops = pairwise_plan(D)

    def leaf(a):
        n = a.shape[1]
        if n < 8:
            r = np.zeros(R, f32)
            for i in range(n):
                r = (r + a[:, i]).astype(f32)
            return r
        r = [a[:, j].astype(f32) for j in range(8)]
        body = n - n % 8
        for i in range(8, body, 8):
            for j in range(8):
                r[j] = (r[j] + a[:, i + j]).astype(f32)
        res = (((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))).astype(f32)
        for i in range(body, n):
            res = (res + a[:, i]).astype(f32)
        return res
    sums = [leaf(sq[:, o:o + n]) for o, n in leaves]
    st, nl = [], 0
    for op in ops:
        if op == 0:
            st.append(sums[nl])
            nl += 1
        else:
            right = st.pop()
            st[-1] = (st[-1] + right).astype(f32)
    total = (f32(0) + st[0]).astype(np.float16)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        nrm = np.sqrt(total.astype(f32)).astype(np.float16)
        return (X.astype(f32) / nrm.astype(f32)[:, None]).astype(np.float16)


def normalize_rows_guarded(F):
    """compare_models.py:1166-1171."""
    n = np.linalg.norm(F, axis=1, keepdims=True)
    n = np.where(n > 1e-8, n, np.ones_like(n))
    return F / n


def search_top_frames_ref(embeddings, text_features, top_k, frames):
    E = normalize_rows(embeddings)
    similarities = np.dot(E, text_features.T).flatten()
    if len(similarities) <= top_k:
        top_indices = np.argsort(similarities)[::-1]
    else:
        top_indices = np.argsort(similarities)[::-1][:top_k]
    pairs = [(frames[i], similarities[i]) for i in top_indices]
    pairs.sort(key=lambda p: p[1], reverse=True)
    return [p[0] for p in pairs], top_indices


def scores_ref(corpus, queries, norm="l2", dtype=np.float64):
    """[Q, N] scores <q, c/|c|> in ``dtype`` (float64 = truth for tolerance checks)."""
    C = np.asarray(corpus, dtype=dtype)
    Qm = np.asarray(queries, dtype=dtype)
    if norm == "l2":
        C = normalize_rows(C)
    elif norm == "l2_guard":
        C = normalize_rows_guarded(C)
    return Qm @ C.T


def topk_ref(corpus, queries, k, index_base=0, norm="l2", nan_policy="first", dtype=np.float64):
    S = np.atleast_2d(scores_ref(corpus, queries, norm, dtype))
    Q, N = S.shape
    kk = min(k, N)
    out_s = np.empty((Q, kk), np.float64)
    out_i = np.empty((Q, kk), np.int64)
    idx = np.arange(N)
    for q in range(Q):
        s = S[q]
        nan = np.isnan(s)
        key = np.where(nan, np.inf if nan_policy == "first" else -np.inf, s)
        # primary: key desc; secondary: index asc (lexsort: last key is primary)
        order = np.lexsort((idx, -key))
        if nan_policy == "first":
            order = np.concatenate([order[nan[order]], order[~nan[order]]])
        else:
            order = np.concatenate([order[~nan[order]], order[nan[order]]])
        out_i[q] = order[:kk] + index_base
        out_s[q] = s[order[:kk]]
    return out_s, out_i


def merge_ref(cand_scores, cand_index, k, nan_policy="first"):
    """Merge [Q, C] candidate lists (index -1 empty) with the same order rule."""
    Q, C = cand_scores.shape
    out_s = np.full((Q, k), -np.inf)
    out_i = np.full((Q, k), -1, np.int64)
    for q in range(Q):
        valid = cand_index[q] >= 0
        s = cand_scores[q][valid].astype(np.float64)
        i = cand_index[q][valid]
        nan = np.isnan(s)
        key = np.where(nan, np.inf if nan_policy == "first" else -np.inf, s)
        order = np.lexsort((i, -key))
        if nan_policy == "first":
            order = np.concatenate([order[nan[order]], order[~nan[order]]])
        else:
            order = np.concatenate([order[~nan[order]], order[nan[order]]])
        n = min(k, len(order))
        out_s[q, :n] = s[order[:n]]
        out_i[q, :n] = i[order[:n]]
    return out_s, out_i


def rank_of_target_ref(s, g):
    """1-based stable rank of s[g] in argsort(-s) (NaN last)."""
    s = np.asarray(s, dtype=np.float64)
    sg = s[g]
    if np.isnan(sg):
        return int((~np.isnan(s)).sum() + np.isnan(s[:g]).sum() + 1)
    return int((s > sg).sum() + (s[:g] == sg).sum() + 1)


def _metrics(ranks):
    ranks = np.asarray(ranks)
    return {"R@1": float((ranks <= 1).mean()), "R@5": float((ranks <= 5).mean()),
            "R@10": float((ranks <= 10).mean()), "MRR": float((1.0 / ranks).mean()),
            "Median_Rank": float(np.median(ranks)), "Mean_Rank": float(np.mean(ranks))}


def retrieval_metrics_ref(image_features, text_features, caption_image_ids, image_ids):
    """compare_models.py:994-1090, literally (np.argsort(-s) per query)."""
    similarity_matrix = np.dot(image_features, text_features.T)
    image_id_to_index = {iid: i for i, iid in enumerate(image_ids)}
    t2i_ranks = []
    for i, iid in enumerate(caption_image_ids):
        if iid in image_id_to_index:
            gt = image_id_to_index[iid]
            sims = similarity_matrix[:, i]
            sorted_indices = np.argsort(-sims)
            t2i_ranks.append(np.where(sorted_indices == gt)[0][0] + 1)
    caps = defaultdict(list)
    for i, iid in enumerate(caption_image_ids):
        caps[iid].append(i)
    i2t_ranks = []
    for j, iid in enumerate(image_ids):
        gt = caps[iid]
        if not gt:
            continue
        sorted_indices = np.argsort(-similarity_matrix[j, :])
        i2t_ranks.append(min(np.where(sorted_indices == idx)[0][0] + 1 for idx in gt))
    t2i = _metrics(t2i_ranks)
    i2t = _metrics(i2t_ranks)
    mean = {m: (t2i[m] + i2t[m]) / 2 for m in t2i}
    mean["rsum"] = t2i["R@1"] + t2i["R@5"] + t2i["R@10"] + i2t["R@1"] + i2t["R@5"] + i2t["R@10"]
    return {"t2i": t2i, "i2t": i2t, "mean": mean,
            "t2i_ranks": np.array(t2i_ranks), "i2t_ranks": np.array(i2t_ranks)}


def assert_topk_equivalent(got_s, got_i, ref_scores_row, k, tol=2e-6, index_base=0, nan_policy="first"):
    """Check a kernel top-k list against float64 truth for one query.

    Exact index equality is required except where the float64 scores of the
    items involved differ by < ``tol`` (near-ties that fp32 summation order may
    legitimately flip; the fixtures assert they do not occur in the pinned
    cases).  Returns the number of tolerated swaps."""
    s = np.asarray(ref_scores_row, dtype=np.float64)
    N = s.shape[0]
    idx = np.arange(N)
    nan = np.isnan(s)
    key = np.where(nan, np.inf if nan_policy == "first" else -np.inf, s)
    order = np.lexsort((idx, -key))
    kk = min(k, N)
    ref = order[:kk] + index_base
    got_i = np.asarray(got_i)[:kk]
    swaps = 0
    for p in range(kk):
        if got_i[p] == ref[p]:
            continue
        a = s[got_i[p] - index_base]
        b = s[ref[p] - index_base]
        if not (abs(a - b) < tol or (np.isnan(a) and np.isnan(b))):
            raise AssertionError(f"position {p}: got index {got_i[p]} (score {a}), expected {ref[p]} (score {b})")
        swaps += 1
    assert len(set(got_i.tolist())) == kk, "duplicate indices in top-k"
    got_s = np.asarray(got_s)[:kk]
    exp_s = s[got_i - index_base]
    fin = ~np.isnan(exp_s)
    assert np.all(np.isnan(got_s[~fin])), "NaN scores must stay NaN"
    assert np.allclose(got_s[fin], exp_s[fin], rtol=0, atol=tol * 4), "score mismatch"
    return swaps
