"""Host image preprocessing: openai/CLIP ``_transform(n_px)`` and the
``compare_models.py`` variant.

  _transform: Resize(n_px, BICUBIC) on the short side -> CenterCrop(n_px) ->
              RGB -> ToTensor -> Normalize(CLIP mean/std)
              (used at Backend/embedding.py:46, embedding_service.py:406,475)
  squash:     Resize((n_px, n_px)) -> ToTensor -> Normalize
              (compare_models.py:387-391)

torchvision is not installed here, so both are restated on PIL + numpy with
torchvision's size arithmetic (short side scaled, long side truncated;
crop offsets rounded).  Host-side like the reference; a GPU decode/resize
kernel is SURVEY.md §8(f) item 1 ("next").
"""
from __future__ import annotations

import numpy as np

MEAN = np.array([0.48145466, 0.4578275, 0.40821073], dtype=np.float32)
STD = np.array([0.26862954, 0.26130258, 0.27577711], dtype=np.float32)


def _to_tensor(img):
    import torch
    a = np.asarray(img.convert("RGB"), dtype=np.float32) / 255.0
    a = (a - MEAN) / STD
    return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))


class Transform:
    def __init__(self, n_px: int, squash: bool = False):
        self.n_px = n_px
        self.squash = squash

    def __call__(self, img):
        from PIL import Image
        n = self.n_px
        if self.squash:
            img = img.resize((n, n), Image.BICUBIC)
            return _to_tensor(img)
        w, h = img.size
        if w <= h:
            nw, nh = n, int(n * h / w)
        else:
            nw, nh = int(n * w / h), n
        if (nw, nh) != (w, h):
            img = img.resize((nw, nh), Image.BICUBIC)
        left = int(round((nw - n) / 2.0))
        top = int(round((nh - n) / 2.0))
        img = img.crop((left, top, left + n, top + n))
        return _to_tensor(img)

    def __repr__(self):
        return f"Transform(n_px={self.n_px}, squash={self.squash})"
