"""miclip — MI355X-native CLIP frame embedding + text->frame retrieval.

The hot path of the reference: openai/CLIP ``encode_image`` /
``encode_text`` and the NumPy ranking of ``EmbeddingService.search_top_frames``,
re-built as gfx950 HIP kernels behind the C-ABI in ``include/miclip.h``.
"""
from .api import available_models, load, tokenize  # noqa: F401
from .config import CLIPConfig, get_config  # noqa: F401
from .model import CLIP  # noqa: F401

__all__ = ["available_models", "load", "tokenize", "CLIP", "CLIPConfig", "get_config"]
