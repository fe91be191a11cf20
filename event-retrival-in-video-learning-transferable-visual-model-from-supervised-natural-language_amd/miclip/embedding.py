"""Standalone folder -> ``.npy`` embedder: mirror of
``Backend/embedding.py:9-59`` ``extract_and_save_embeddings_from_folder``
(BASELINE.json configs[0]'s flow).

Same device choice (``"cuda" if torch.cuda.is_available() else "cpu"``,
embedding.py:21 — on a CPU-only host ``clip.load`` then raises, since this
framework has no CPU execution path), same walk order (``os.walk``, files in
directory order, embedding.py:39-43), same extensions, same UN-normalised rows
(embedding.py:48-56), same ``{video_name}_embeddings.npy`` naming, and an
unreadable image raises as ``Image.open`` does in the reference.  The
reference encodes one image per call and hard-codes a Windows output
directory; here frames are decoded on host threads, resized/cropped/normalised
on the GPU (Pillow-exact, ``preprocess.load_frames``) and encoded in batches
(results are per frame, so batching does not change them), and
``output_dir`` is a parameter (default ``./embedding``).  Rows are float32
(the reference's CPU path; its CUDA path stores the fp16 model's output).
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np

from . import api
from .preprocess import Transform, decode_chunk, load_frames


def walk_frames(folder_path):
    """Image paths in the reference's order (embedding.py:39-43)."""
    paths = []
    for root, _, files in os.walk(folder_path):
        for file in files:
            if file.lower().endswith((".jpg", ".jpeg", ".png")):
                paths.append(os.path.join(root, file))
    return paths


def extract_and_save_embeddings_from_folder(folder_path, model_name, video_name=None, output_dir="embedding",
                                            batch_size=256, model=None, preprocess=None, weights="bf16"):
    """``weights="fp32"`` runs the reference's CPU arithmetic (configs[0]: the
    fp32 model ``clip.load`` builds on a CPU) on the fp32 tower."""
    import torch
    from PIL import Image

    if model is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
        model, preprocess = api.load(model_name, device=device, weights=weights)
    os.makedirs(output_dir, exist_ok=True)
    if not video_name:
        video_name = Path(folder_path).name
    output_file = os.path.join(output_dir, f"{video_name}_embeddings.npy")
    paths = walk_frames(folder_path)
    rows = []
    gpu_prep = isinstance(preprocess, Transform)   # this package's transform: GPU decode/resize/crop/normalise
    step = decode_chunk(batch_size) if gpu_prep else batch_size
    for j in range(0, len(paths), step):
        if gpu_prep:
            frames, _ = load_frames(paths[j:j + step], preprocess.n_px, device=model.device,
                                    squash=preprocess.squash, strict=True)
        for i in range(0, min(step, len(paths) - j), batch_size):
            if gpu_prep:
                batch = frames[i:i + batch_size]
            else:
                batch = torch.stack([preprocess(Image.open(p).convert("RGB")) for p in paths[j + i:j + i + batch_size]])
            rows.append(model.encode_image(batch, out_dtype=torch.float32).cpu().numpy())
    all_embeddings = np.vstack(rows) if rows else np.zeros((0, model.visual.output_dim), np.float32)
    np.save(output_file, all_embeddings)
    return output_file
