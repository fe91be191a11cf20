"""``clip`` module surface: ``load``, ``tokenize``, ``available_models``.

Drop-in for the third-party openai/CLIP calls the reference makes:
``clip.load("ViT-B/32", device)`` (Backend/embedding.py:22,
Backend/services/embedding_service.py:86,106, compare_models.py:316) and
``clip.tokenize`` (embedding_service.py:169, compare_models.py:1202).
"""
from __future__ import annotations

from . import _native, config
from . import weights as _weights
from .model import CLIP
from .preprocess import Transform
from .tokenizer import tokenize  # noqa: F401


def available_models():
    return config.available_models()


def load(name, device=None, jit=False, download_root=None, image_chunk=None, weights="bf16"):
    """Returns ``(model, preprocess)`` like openai/CLIP.

    ``name`` is a model name (weights from the local ``$CLIP_WEIGHTS``
    checkpoint; random-init weights only when explicitly requested, see
    ``weights.resolve``) or a path to a local OpenAI checkpoint.  There is no
    download (no network) and no JIT: ``jit`` and ``download_root`` are
    accepted for signature compatibility.  ``weights="fp8"`` selects the MX-fp8
    vision GEMMs (BASELINE.json configs[4]).

    Device policy: the reference picks ``"cuda" if torch.cuda.is_available()
    else "cpu"`` (Backend/embedding.py:21, embedding_service.py:70), which on
    the MI355X host is ``"cuda"`` (ROCm's torch device name).  ``device="cpu"``
    raises: this framework has no CPU execution path, and the CPU restatement
    under ``oracle/`` is test infrastructure (the parity checker and the
    benchmark's CPU baseline), never a fallback for the product.
    """
    import torch
    if device is None:
        device = "cuda"
    dev = torch.device(device)
    if dev.type != "cuda":
        raise _native.MiClipError(
            f"clip.load(device={device!r}): miclip runs only on the GPU (device 'cuda' on ROCm, MI355X); there is "
            "no CPU execution path and the CPU restatement in oracle/ is test infrastructure, not a fallback")
    cfg, sd = _weights.resolve(name)
    model = CLIP(cfg, sd, device=dev, image_chunk=image_chunk, weights=weights)
    return model, Transform(cfg.image_resolution)
