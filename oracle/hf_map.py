"""ORACLE (test infrastructure only) — build the in-container HF ``CLIPModel``
(transformers 5.15.0, ``models/clip/modeling_clip.py``) from an OpenAI-layout
state dict.  This is the architecture pin for ``clip_ref``: openai/CLIP itself
is absent.

OpenAI -> HF mapping: ``in_proj_weight`` splits into q/k/v,
``visual.proj`` / ``text_projection`` are applied as ``x @ P`` so the HF linear
weight is ``P.T``, ``ln_pre`` -> ``pre_layrnorm``, ``conv1`` ->
``patch_embedding``; text pooling uses ``eos_token_id=2`` (argmax rule).
"""
from __future__ import annotations

import numpy as np


def build_hf(sd, cfg):
    import torch
    from transformers import CLIPConfig as HFConfig, CLIPModel

    hf_cfg = HFConfig(
        text_config=dict(vocab_size=cfg.vocab_size, hidden_size=cfg.text_width,
                         intermediate_size=4 * cfg.text_width, num_hidden_layers=cfg.text_layers,
                         num_attention_heads=cfg.text_heads, max_position_embeddings=cfg.context_length,
                         hidden_act="quick_gelu", layer_norm_eps=1e-5, eos_token_id=2,
                         projection_dim=cfg.embed_dim),
        vision_config=dict(hidden_size=cfg.vision_width, intermediate_size=4 * cfg.vision_width,
                           num_hidden_layers=cfg.vision_layers, num_attention_heads=cfg.vision_heads,
                           image_size=cfg.image_resolution, patch_size=cfg.vision_patch_size,
                           hidden_act="quick_gelu", layer_norm_eps=1e-5, projection_dim=cfg.embed_dim),
        projection_dim=cfg.embed_dim,
    )
    hf_cfg._attn_implementation = "eager"
    model = CLIPModel(hf_cfg).eval()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))  # noqa: E731
    new = {}

    def tower(src, dst, width, layers):
        for i in range(layers):
            s, d = f"{src}resblocks.{i}.", f"{dst}encoder.layers.{i}."
            w = sd[s + "attn.in_proj_weight"]
            b = sd[s + "attn.in_proj_bias"]
            for j, n in enumerate(("q", "k", "v")):
                new[d + f"self_attn.{n}_proj.weight"] = t(w[j * width:(j + 1) * width])
                new[d + f"self_attn.{n}_proj.bias"] = t(b[j * width:(j + 1) * width])
            new[d + "self_attn.out_proj.weight"] = t(sd[s + "attn.out_proj.weight"])
            new[d + "self_attn.out_proj.bias"] = t(sd[s + "attn.out_proj.bias"])
            new[d + "layer_norm1.weight"] = t(sd[s + "ln_1.weight"])
            new[d + "layer_norm1.bias"] = t(sd[s + "ln_1.bias"])
            new[d + "layer_norm2.weight"] = t(sd[s + "ln_2.weight"])
            new[d + "layer_norm2.bias"] = t(sd[s + "ln_2.bias"])
            new[d + "mlp.fc1.weight"] = t(sd[s + "mlp.c_fc.weight"])
            new[d + "mlp.fc1.bias"] = t(sd[s + "mlp.c_fc.bias"])
            new[d + "mlp.fc2.weight"] = t(sd[s + "mlp.c_proj.weight"])
            new[d + "mlp.fc2.bias"] = t(sd[s + "mlp.c_proj.bias"])

    v = "vision_model."
    new[v + "embeddings.class_embedding"] = t(sd["visual.class_embedding"])
    new[v + "embeddings.patch_embedding.weight"] = t(sd["visual.conv1.weight"])
    new[v + "embeddings.position_embedding.weight"] = t(sd["visual.positional_embedding"])
    new[v + "pre_layrnorm.weight"] = t(sd["visual.ln_pre.weight"])
    new[v + "pre_layrnorm.bias"] = t(sd["visual.ln_pre.bias"])
    new[v + "post_layernorm.weight"] = t(sd["visual.ln_post.weight"])
    new[v + "post_layernorm.bias"] = t(sd["visual.ln_post.bias"])
    tower("visual.transformer.", v, cfg.vision_width, cfg.vision_layers)
    tm = "text_model."
    new[tm + "embeddings.token_embedding.weight"] = t(sd["token_embedding.weight"])
    new[tm + "embeddings.position_embedding.weight"] = t(sd["positional_embedding"])
    new[tm + "final_layer_norm.weight"] = t(sd["ln_final.weight"])
    new[tm + "final_layer_norm.bias"] = t(sd["ln_final.bias"])
    tower("transformer.", tm, cfg.text_width, cfg.text_layers)
    new["visual_projection.weight"] = t(sd["visual.proj"].T)
    new["text_projection.weight"] = t(sd["text_projection"].T)
    new["logit_scale"] = t(sd["logit_scale"])
    missing, unexpected = model.load_state_dict(new, strict=False)
    missing = [m for m in missing if not m.endswith("position_ids")]
    if missing or unexpected:
        raise RuntimeError(f"HF mapping mismatch: missing={missing} unexpected={unexpected}")
    return model


def hf_encode(model, pixels=None, tokens=None):
    import torch
    with torch.no_grad():
        out = {}
        if pixels is not None:
            out["image"] = model.get_image_features(pixel_values=torch.from_numpy(pixels))
        if tokens is not None:
            out["text"] = model.get_text_features(input_ids=torch.from_numpy(np.asarray(tokens, dtype=np.int64)))
    res = {}
    for k, v in out.items():
        if not isinstance(v, torch.Tensor):
            v = v.pooler_output
        res[k] = v.numpy()
    return res
