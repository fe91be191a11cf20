"""ORACLE (test infrastructure only) — numpy restatement of the image
preprocessing the reference runs on the host before ``encode_image``.

Reference call sites: openai/CLIP ``preprocess = _transform(n_px)`` =
``Resize(n_px, BICUBIC)`` (short side) -> ``CenterCrop(n_px)`` -> RGB ->
``ToTensor`` -> ``Normalize(CLIP mean/std)``, applied per frame at
``Backend/embedding.py:46`` and ``Backend/services/embedding_service.py:406,475``;
and ``compare_models.py:387-391`` ``Resize((224, 224))`` (torchvision's
default BILINEAR) -> ``ToTensor`` -> ``Normalize``.  torchvision hands PIL
images to Pillow's ``Image.resize``, i.e. Pillow's ``ImagingResample``
(``libImaging/Resample.c``; Pillow 12.2 in this image), restated here:

  * separable, horizontal pass first, then vertical;
  * per output index: center = (i + 0.5) * scale, filter support scaled by
    max(scale, 1) (antialiasing when downscaling), taps
    [int(center - support + 0.5), int(center + support + 0.5)) clipped to the
    input, weights filter((j - center + 0.5) / max(scale, 1)) normalised to
    sum 1 in double;
  * 8-bit path: weights quantised to int32 with 22 fractional bits
    (round half away from zero), accumulator starts at 2^21, result
    (acc >> 22) clamped to [0, 255] -> uint8 after EACH pass.

Pinned bit-exactly against PIL itself (``tests/test_preprocess.py``); the
HIP kernels (``csrc/preprocess.hip``) are checked against PIL and this file.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2
MEAN = np.array([0.48145466, 0.4578275, 0.40821073], dtype=np.float32)
STD = np.array([0.26862954, 0.26130258, 0.27577711], dtype=np.float32)

BICUBIC, BILINEAR = 0, 1


def _bicubic(x):
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def _bilinear(x):
    x = abs(x)
    return 1.0 - x if x < 1.0 else 0.0


FILTERS = {BICUBIC: (_bicubic, 2.0), BILINEAR: (_bilinear, 1.0)}


def coeffs(in_size, out_size, filt=BICUBIC, in0=0.0, in1=None):
    """Pillow precompute_coeffs + normalize_coeffs_8bpc: (int32 [out, ksize], bounds [out, 2])."""
    fn, fsupport = FILTERS[filt]
    if in1 is None:
        in1 = float(in_size)
    scale = filterscale = float(np.float32(in1) - np.float32(in0)) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = fsupport * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    kk = np.zeros((out_size, ksize), np.int32)
    bounds = np.zeros((out_size, 2), np.int32)
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        w = [fn((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        if ww != 0.0:
            w = [v / ww for v in w]
        for x, v in enumerate(w):
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return kk, bounds


def _pass(src, kk, bounds, axis):
    """One 8-bit pass along `axis` of an HxWxC uint8 array."""
    s = np.moveaxis(src.astype(np.int64), axis, 0)
    out = np.empty((kk.shape[0],) + s.shape[1:], np.uint8)
    for i in range(kk.shape[0]):
        lo, n = bounds[i]
        acc = np.full(s.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for j in range(n):
            acc += s[lo + j] * int(kk[i, j])
        out[i] = np.clip(acc >> PRECISION_BITS, 0, 255)
    return np.moveaxis(out, 0, axis)


def resize(img, size, filt=BICUBIC):
    """PIL ``Image.resize((w, h), filter)`` on an HxWx3 uint8 array."""
    h, w = img.shape[:2]
    ow, oh = size
    if (ow, oh) == (w, h):
        return img.copy()
    out = img
    if ow != w:
        kh, bh = coeffs(w, ow, filt)
        out = _pass(out, kh, bh, 1)
    if oh != h:
        kv, bv = coeffs(h, oh, filt)
        out = _pass(out, kv, bv, 0)
    return out


def clip_transform_geometry(w, h, n):
    """torchvision Resize(n) (short side) + CenterCrop(n) arithmetic:
    resized (nw, nh) and crop (left, top)."""
    if w <= h:
        nw, nh = n, int(n * h / w)
    else:
        nw, nh = int(n * w / h), n
    return nw, nh, int(round((nw - n) / 2.0)), int(round((nh - n) / 2.0))


def to_tensor_normalize(u8):
    a = u8.astype(np.float32) / np.float32(255.0)
    return ((a - MEAN) / STD).transpose(2, 0, 1).astype(np.float32)


def clip_transform(img, n=224):
    """openai/CLIP _transform(n) on an HxWx3 uint8 RGB array -> [3, n, n] f32."""
    h, w = img.shape[:2]
    nw, nh, left, top = clip_transform_geometry(w, h, n)
    r = resize(img, (nw, nh), BICUBIC)
    return to_tensor_normalize(r[top:top + n, left:left + n])


def squash_transform(img, n=224):
    """compare_models.py:387-391: Resize((n, n)) (bilinear) -> ToTensor -> Normalize."""
    return to_tensor_normalize(resize(img, (n, n), BILINEAR))
