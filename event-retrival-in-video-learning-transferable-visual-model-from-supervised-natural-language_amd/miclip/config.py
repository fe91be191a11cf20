"""CLIP architecture descriptions.

The reference never builds a model itself: it calls the third-party
openai/CLIP ``clip.load(name, device)`` (call sites
``Backend/embedding.py:22``, ``Backend/services/embedding_service.py:86,106``,
``Backend/content/Test_compare_model/compare_models.py:316``).  openai/CLIP's
``build_model`` infers every dimension from the OpenAI state dict; this module
restates that inference (``from_state_dict``) and names the published ViT
variants the survey scopes (ViT-B/32, ViT-L/14,
ViT-L/14@336px; ViT-B/16 is the same family).
"""
from __future__ import annotations

from dataclasses import dataclass, asdict


@dataclass(frozen=True)
class CLIPConfig:
    name: str
    embed_dim: int            # joint embedding dimension D (512 / 768)
    image_resolution: int     # R
    vision_layers: int
    vision_width: int
    vision_patch_size: int
    context_length: int       # 77
    vocab_size: int           # 49408
    text_width: int
    text_heads: int
    text_layers: int

    @property
    def vision_heads(self) -> int:
        return self.vision_width // 64

    @property
    def grid(self) -> int:
        return self.image_resolution // self.vision_patch_size

    @property
    def vision_tokens(self) -> int:
        return self.grid * self.grid + 1

    @property
    def patch_k(self) -> int:
        return 3 * self.vision_patch_size * self.vision_patch_size

    def as_dict(self):
        return asdict(self)

    # ---- algorithmic work (what roofline.achieved is computed from) ----
    def image_flops(self) -> float:
        """Dense FLOPs of one encode_image frame (2 x MACs); SURVEY.md §8(d)."""
        W, S, L = self.vision_width, self.vision_tokens, self.vision_layers
        g2 = self.grid * self.grid
        f = 2.0 * g2 * self.patch_k * W                      # patch embed
        per_layer = 2.0 * S * W * (3 * W + W + 4 * W + 4 * W)  # qkv, out, fc, proj
        per_layer += 2.0 * 2.0 * S * S * W                    # QK^T and PV
        f += L * per_layer
        f += 2.0 * W * self.embed_dim                        # CLS projection
        return f

    def image_attention_flops(self, last_query_rows: int | None = None) -> float:
        """QK^T and PV of all layers per frame; ``last_query_rows``: the query rows the last
        layer's attention computes (the CLS-row last block computes the CLS query's tile only)."""
        W, S, L = self.vision_width, self.vision_tokens, self.vision_layers
        r = S if last_query_rows is None else min(S, last_query_rows)
        return 4.0 * S * S * W * (L - 1) + 4.0 * r * S * W

    def image_flops_executed(self, cls_last: bool = True, q_cls: bool = False,
                             last_query_rows: int | None = None) -> float:
        """image_flops less the work the last block skips when it runs its row-wise part on the
        CLS rows only (api.cpp last_block_cls / run_tower_mx: out_proj, c_fc and c_proj for S - 1
        of S rows per frame; their outputs are never read); ``q_cls``: its in_proj also computes Q
        for the CLS rows only (the LN-folded bf16 and the fp32 towers; 2 (S - 1) W^2 less);
        ``last_query_rows``: its attention computes that many query rows (the CLS query's tile)."""
        W, S = self.vision_width, self.vision_tokens
        f = self.image_flops()
        if cls_last:
            f -= 2.0 * (S - 1) * W * (W + 4 * W + 4 * W)
        if q_cls:
            f -= 2.0 * (S - 1) * W * W
        return f - (self.image_attention_flops() - self.image_attention_flops(last_query_rows))

    def text_attention_flops(self) -> float:
        return 4.0 * self.context_length * self.context_length * self.text_width * self.text_layers

    def text_flops(self) -> float:
        W, S, L = self.text_width, self.context_length, self.text_layers
        per_layer = 2.0 * S * W * 12 * W + 2.0 * 2.0 * S * S * W
        return L * per_layer + 2.0 * W * self.embed_dim


_MODELS = {
    "ViT-B/32": CLIPConfig("ViT-B/32", 512, 224, 12, 768, 32, 77, 49408, 512, 8, 12),
    "ViT-B/16": CLIPConfig("ViT-B/16", 512, 224, 12, 768, 16, 77, 49408, 512, 8, 12),
    "ViT-L/14": CLIPConfig("ViT-L/14", 768, 224, 24, 1024, 14, 77, 49408, 768, 12, 12),
    "ViT-L/14@336px": CLIPConfig("ViT-L/14@336px", 768, 336, 24, 1024, 14, 77, 49408, 768, 12, 12),
    # small configurations used only by the parity tests (same code path)
    "test-tiny": CLIPConfig("test-tiny", 128, 64, 2, 128, 16, 77, 1000, 128, 2, 2),
    "test-small": CLIPConfig("test-small", 256, 96, 3, 256, 32, 77, 2000, 256, 4, 2),
}


def available_models():
    """Mirror of ``clip.available_models()`` restricted to the ViT family."""
    return [k for k in _MODELS if not k.startswith("test-")]


def get_config(name: str) -> CLIPConfig:
    if name not in _MODELS:
        raise RuntimeError(f"Model {name} not found; available models = {list(_MODELS)}")
    return _MODELS[name]


def from_state_dict(sd, name: str = "custom") -> CLIPConfig:
    """Infer the architecture from an OpenAI-layout state dict (openai/CLIP
    ``build_model``; the reference reaches it through ``clip.load(..., jit=False)``
    at ``embedding_service.py:106``)."""
    if "visual.proj" not in sd:
        raise RuntimeError("only ViT CLIP state dicts are supported (no 'visual.proj' key)")
    vision_width = sd["visual.conv1.weight"].shape[0]
    vision_layers = len([k for k in sd if k.startswith("visual.") and k.endswith(".attn.in_proj_weight")])
    vision_patch = sd["visual.conv1.weight"].shape[-1]
    grid = round((sd["visual.positional_embedding"].shape[0] - 1) ** 0.5)
    embed_dim = sd["text_projection"].shape[1]
    ctx = sd["positional_embedding"].shape[0]
    vocab = sd["token_embedding.weight"].shape[0]
    tw = sd["ln_final.weight"].shape[0]
    tl = len({k.split(".")[2] for k in sd if k.startswith("transformer.resblocks")})
    for known in _MODELS.values():
        if (known.vision_width, known.vision_layers, known.vision_patch_size, known.grid,
                known.embed_dim, known.text_width, known.text_layers) == (
                vision_width, vision_layers, vision_patch, grid, embed_dim, tw, tl):
            name = known.name
            break
    return CLIPConfig(name, embed_dim, vision_patch * grid, vision_layers, vision_width, vision_patch,
                      ctx, vocab, tw, tw // 64, tl)
