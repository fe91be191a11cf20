"""``clip`` module surface: ``load``, ``tokenize``, ``available_models``.

Drop-in for the third-party openai/CLIP calls the reference makes:
``clip.load("ViT-B/32", device)`` (Backend/embedding.py:22,
Backend/services/embedding_service.py:86,106, compare_models.py:316) and
``clip.tokenize`` (embedding_service.py:169, compare_models.py:1202).
"""
from __future__ import annotations

from . import config
from . import weights as _weights
from .model import CLIP
from .preprocess import Transform
from .tokenizer import tokenize  # noqa: F401


def available_models():
    return config.available_models()


def load(name, device=None, jit=False, download_root=None, image_chunk=None, weights="bf16"):
    """Returns ``(model, preprocess)`` like openai/CLIP.

    ``name`` is a model name (deterministic random-init weights, or the local
    ``$CLIP_WEIGHTS`` checkpoint when it matches) or a path to a local OpenAI
    checkpoint.  There is no download (no network) and no JIT: ``jit`` and
    ``download_root`` are accepted for signature compatibility.  ``weights="fp8"``
    selects the MX-fp8 vision GEMMs (BASELINE.json configs[4]).
    """
    import torch
    if device is None:
        device = "cuda"
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError("miclip runs on MI355X (device 'cuda' on ROCm); no CPU execution path")
    cfg, sd = _weights.resolve(name)
    model = CLIP(cfg, sd, device=dev, image_chunk=image_chunk, weights=weights)
    return model, Transform(cfg.image_resolution)
