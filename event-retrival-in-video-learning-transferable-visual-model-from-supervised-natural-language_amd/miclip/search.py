"""``SearchService.search_by_image`` (``Backend/services/search_service.py:611-706``)
on the GPU path, without the per-candidate re-encode.

The reference encodes the query image, takes ``top_k * 3`` candidates from
``EmbeddingService.search_top_frames_by_image``, and then, for EVERY candidate,
re-reads the frame from disk and re-encodes it (``extract_image_embedding``,
``embedding_service.py:394-420``: one PIL decode + one encode_image call per
frame) only to recompute the cosine the ranking has just computed.  Here the
candidates and their cosines come from one ``mi_rank_topk`` pass over the
HBM-resident corpus (the stored rows are the encoder's own output, normalised
in the rank kernel exactly as ``extract_image_embedding`` normalises), so the
loop does no I/O.  ``reencode=True`` keeps the reference's re-encode semantics
for corpora whose stored rows did not come from the active model, but batches
the candidates into one GPU encode instead of one call per frame.

Everything else follows the reference: the three image sources (http(s) URL,
``data:image`` URL, local path — the ``data:image`` branch hands the base64
TEXT to PIL without decoding it, so it always fails into the outer
``except`` and returns ``[]``, as there), the finetuned / original model
switch, the first metadata row whose ``frameidx`` equals the candidate's stem
(``next(...)``, :672, here one dict built per call instead of a scan per
candidate), ``similarity >= adaptive_threshold``, the event fields
``clip_similarity`` and ``confidence``, a stable sort by ``clip_similarity``
descending and ``[:top_k]``; per-candidate errors are printed and skipped, any
other error prints and returns ``[]``.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np


def load_query_image(image_url):
    """search_service.py:630-642: the three image sources, RGB."""
    from io import BytesIO

    from PIL import Image
    if image_url.startswith(("http://", "https://")):
        import requests   # network fetch: a deployment concern, not the hot path
        response = requests.get(image_url)
        return Image.open(BytesIO(response.content)).convert("RGB")
    if image_url.startswith("data:image"):
        encoded_data = image_url.split(",")[1]
        return Image.open(BytesIO(bytes(encoded_data, "utf-8"))).convert("RGB")   # as the reference (no b64decode)
    return Image.open(image_url).convert("RGB")


def _encode(embedding_service, x):
    """One batch through the active model, L2-normalised rows (search_service.py:649-658)."""
    import torch
    if embedding_service.get_active_model_name() == "finetuned" and embedding_service.finetuned_model is not None:
        f = embedding_service.finetuned_model(x)
    else:
        f = embedding_service.original_model.encode_image(x, normalize=False, out_dtype=torch.float32)
    f = f.float()
    return (f / f.norm(dim=-1, keepdim=True)).cpu().numpy()


def _reencode(embedding_service, frame_names, preprocess):
    """The reference's per-candidate extract_image_embedding, batched: one
    host decode + preprocess per frame, ONE encode; None for unreadable frames."""
    import torch
    from PIL import Image
    xs, ok = [], []
    for name in frame_names:
        try:
            xs.append(preprocess(Image.open(name)))
            ok.append(True)
        except Exception as e:
            print(f"Error extracting embedding from {name}: {e}")
            ok.append(False)
    out = [None] * len(frame_names)
    if xs:
        feats = _encode(embedding_service, torch.stack(xs))
        it = iter(feats)
        for j, good in enumerate(ok):
            if good:
                out[j] = next(it)[None, :]
    return out


def search_by_image(embedding_service, data_service, image_url, adaptive_threshold, top_k, video_name=None,
                    preprocess=None, reencode=False, data=None):
    """search_service.py:611-706 with the reference's arguments; ``data_service``
    provides ``load_json_data(video_name)`` and ``format_event_for_frontend(row)``
    as the reference's DataService does (``data`` may be passed directly)."""
    try:
        img = load_query_image(image_url)
        if preprocess is None:
            preprocess = embedding_service.preprocess
        image = preprocess(img).unsqueeze(0)
        image_features = _encode(embedding_service, image)                    # [1, D], normalised

        # candidates and their cosines in one fused pass (search_top_frames_by_image, top_k * 3)
        corpus = embedding_service._corpus_on_device(video_name)
        if corpus is None:
            similar, scores = [], np.zeros(0, np.float32)
        else:
            scores, idx = embedding_service._rank(corpus, image_features.reshape(-1), top_k * 3)
            frames = embedding_service._frames(video_name)
            similar = [frames[i] for i in idx]

        if data is None:
            data = data_service.load_json_data(video_name)
        first = {}
        for item in data:
            fi = item.get("frameidx")
            if fi is not None and fi not in first:
                first[fi] = item
        fresh = _reencode(embedding_service, similar, preprocess) if reencode else None

        results = []
        for j, frame_name in enumerate(similar):
            try:
                frame_idx = int(Path(frame_name).stem)
                frame_data = first.get(frame_idx)
                if frame_data:
                    if reencode:
                        emb = fresh[j]
                        if emb is None:
                            continue
                        similarity = float(np.dot(emb, image_features.T)[0][0])
                    else:
                        similarity = float(scores[j])
                    if similarity >= adaptive_threshold:
                        frame_data_copy = frame_data.copy()
                        frame_data_copy["clip_similarity"] = similarity
                        event = data_service.format_event_for_frontend(frame_data_copy)
                        event["clip_similarity"] = similarity
                        event["confidence"] = similarity
                        results.append(event)
            except Exception as e:
                print(f"Error processing frame {frame_name}: {e}")
        results.sort(key=lambda x: x.get("clip_similarity", 0), reverse=True)
        return results[:top_k]
    except Exception as e:
        print(f"Error in image search: {e}")
        return []
