"""Drop-in ``clip`` module (openai/CLIP surface) backed by miclip's HIP path.

With this package directory on ``sys.path`` the reference's own call sites —
``import clip; model, preprocess = clip.load("ViT-B/32", device)``,
``clip.tokenize(...)``, ``model.encode_image`` / ``model.encode_text``
(Backend/embedding.py:3,22,46-49; Backend/services/embedding_service.py:8,86,169-177)
— run unchanged on MI355X.
"""
from miclip.api import available_models, load, tokenize  # noqa: F401
from miclip.model import CLIP  # noqa: F401

__all__ = ["available_models", "load", "tokenize"]
