"""R@K retrieval evaluation — the CLIP branch of
``ModelComparison.evaluate_model`` (Backend/content/Test_compare_model/compare_models.py:908-1100).

  S = image_features @ text_features.T                                   :999
  t2i: per caption i, rank of its image in argsort(-S[:, i]) (1-based)   :1004-1016
  i2t: per image j, min rank of its captions in argsort(-S[j, :])        :1045-1062
  R@1/5/10 = mean(rank <= K), MRR, Median_Rank, Mean_Rank                :1020-1027, 1066-1073
  mean over directions, rsum = sum of the six recalls                     :1082-1088

The similarity matrix and the ranks are computed on the GPU
(``mi_score_matrix`` fp32-exact products, ``mi_rank_of_targets`` =
1 + #{greater} + #{equal with lower index}, the stable-sort tie rule); the
final averages are host reductions over 5-6k integers.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np

from . import retrieval


def normalize_guarded(features):
    """``norms = where(norm > 1e-8, norm, 1); f / norms`` (compare_models.py:1166-1171, 1254-1259)."""
    import torch
    n = features.float().norm(dim=1, keepdim=True)
    n = torch.where(n > 1e-8, n, torch.ones_like(n))
    return features.float() / n


def _metrics(ranks):
    ranks = np.asarray(ranks)
    return {
        "R@1": float((ranks <= 1).mean()),
        "R@5": float((ranks <= 5).mean()),
        "R@10": float((ranks <= 10).mean()),
        "MRR": float((1.0 / ranks).mean()),
        "Median_Rank": float(np.median(ranks)),
        "Mean_Rank": float(np.mean(ranks)),
    }


def retrieval_metrics(image_features, text_features, caption_image_ids, image_ids):
    """image_features [I,D], text_features [T,D] (device, already normalised as
    in process_image_batch / process_text_batch); caption_image_ids[t] = image id
    of caption t; image_ids[j] = id of image row j."""
    img = image_features.float().contiguous()
    txt = text_features.float().contiguous()
    id_to_index = {iid: j for j, iid in enumerate(image_ids)}

    # t2i: queries = captions, corpus = images
    pq, pt = [], []
    for i, iid in enumerate(caption_image_ids):
        if iid in id_to_index:
            pq.append(i)
            pt.append(id_to_index[iid])
    s_t2i = retrieval.score_matrix(img, txt, norm="none")            # [T, I]
    t2i_ranks = retrieval.rank_of_targets(s_t2i, pq, pt).cpu().numpy() if pq else np.zeros(0, np.int64)

    # i2t: queries = images, corpus = captions
    caps = defaultdict(list)
    for i, iid in enumerate(caption_image_ids):
        caps[iid].append(i)
    pq2, pt2, owner = [], [], []
    for j, iid in enumerate(image_ids):
        for i in caps.get(iid, []):
            pq2.append(j)
            pt2.append(i)
            owner.append(j)
    s_i2t = retrieval.score_matrix(txt, img, norm="none")            # [I, T]
    r = retrieval.rank_of_targets(s_i2t, pq2, pt2).cpu().numpy() if pq2 else np.zeros(0, np.int64)
    best = {}
    for j, rank in zip(owner, r):
        best[j] = min(best.get(j, rank), rank)
    i2t_ranks = np.array([best[j] for j in sorted(best)], dtype=np.int64)

    t2i = _metrics(t2i_ranks)
    i2t = _metrics(i2t_ranks)
    mean = {m: (t2i[m] + i2t[m]) / 2 for m in t2i}
    mean["rsum"] = t2i["R@1"] + t2i["R@5"] + t2i["R@10"] + i2t["R@1"] + i2t["R@5"] + i2t["R@10"]
    return {"t2i": t2i, "i2t": i2t, "mean": mean, "t2i_ranks": t2i_ranks, "i2t_ranks": i2t_ranks}
