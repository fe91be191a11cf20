"""R@K retrieval evaluation — the CLIP branch of
``ModelComparison.evaluate_model`` (Backend/content/Test_compare_model/compare_models.py:908-1100).

  images -> encode_image -> guarded L2 (process_image_batch)             :938-945, :1102-1173
  captions -> clip.tokenize(truncate=True) -> encode_text -> guarded L2  :980-989, :1190-1261
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

import os
import time
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


def encode_images(model, images, batch_size=32):
    """process_image_batch over the whole set (compare_models.py:938-945,
    1102-1173): ``encode_image`` then the guarded L2 (fused in the kernel,
    ``normalize="guarded"``).  ``images`` is a [I,3,R,R] tensor in dataset order
    (the DataLoader's output) or a list of image files, decoded and squash-resized
    on the GPU (``Resize((R, R))`` + ``Normalize``, :387-391).  Rows do not
    depend on how frames are batched, so the set is encoded in the context's
    chunks; ``batch_size`` is the reference's (32) and only sizes file loads."""
    import torch
    from .preprocess import decode_chunk, load_frames
    if isinstance(images, (list, tuple)) and (not images or isinstance(images[0], (str, os.PathLike))):
        R = model.cfg.image_resolution
        feats = []
        step = decode_chunk(batch_size)
        for j in range(0, len(images), step):
            x, _ = load_frames([str(p) for p in images[j:j + step]], R, device=model.device, squash=True)
            feats.append(model.encode_image(x, normalize="guarded", out_dtype=torch.float32))
        return torch.cat(feats) if feats else torch.zeros(0, model.visual.output_dim, device=model.device)
    return model.encode_image(images, normalize="guarded", out_dtype=torch.float32)


def encode_captions(model, captions):
    """process_text_batch (compare_models.py:980-989, 1190-1261):
    ``clip.tokenize(captions, truncate=True)`` -> ``encode_text`` -> guarded L2.
    ``captions``: list of str, or an int tensor / array of token rows already
    in clip.tokenize format (the BPE vocabulary is not available offline)."""
    import torch
    from . import api
    if isinstance(captions, (list, tuple)) and (not captions or isinstance(captions[0], str)):
        tokens = api.tokenize(list(captions), truncate=True)
    else:
        tokens = captions if isinstance(captions, torch.Tensor) else torch.as_tensor(np.asarray(captions))
    return model.encode_text(tokens, normalize="guarded", out_dtype=torch.float32)


def evaluate_model(model, images, captions, caption_image_ids, image_ids, batch_size=32):
    """``ModelComparison.evaluate_model`` for a CLIP model of this package
    (compare_models.py:908-1100): encode every image and caption, then the t2i /
    i2t ranks and metrics of ``retrieval_metrics``.  Returns the reference's
    ``{'t2i', 'i2t', 'mean', 'processing_time'}`` plus the ranks and the
    features.  Run it on a ``weights="fp32"`` model (or after ``model.float()``)
    for the reference's fp32 arithmetic: ranks and R@1/5/10 then match the
    reference's CPU flow wherever its decisive score gaps exceed f32 rounding
    (tests/test_gpu_rk_flow.py)."""
    import torch
    dev = model.device
    t0 = time.time()
    img = encode_images(model, images, batch_size)
    torch.cuda.synchronize(dev)
    t1 = time.time()
    txt = encode_captions(model, captions)
    torch.cuda.synchronize(dev)
    t2 = time.time()
    res = retrieval_metrics(img, txt, list(caption_image_ids), list(image_ids))
    t3 = time.time()
    res["processing_time"] = t3 - t0
    res["times"] = {"encode_image": t1 - t0, "encode_text": t2 - t1, "rank": t3 - t2}
    res["image_features"], res["text_features"] = img, txt
    return res
