"""ORACLE (test infrastructure only) — numpy restatement of openai/CLIP inference.

The reference calls ``model.encode_image`` / ``model.encode_text`` of the
third-party openai/CLIP package (``Backend/embedding.py:49``,
``Backend/services/embedding_service.py:174,177,490``,
``compare_models.py:1118,1204``).  That package is not vendored
(``Backend/CLIP/`` is empty, ``.gitignore:8``), so the algorithm is restated
from its published ``model.py`` semantics, cross-checked line by line with the
in-container HF equivalent
``transformers/models/clip/modeling_clip.py`` (embeddings :202-218,
attention :280-335, MLP :338-350, pre-LN layer :353-388, text argmax pooling
:559-571, vision CLS pooling + post-LN :641-651, bias-free projections
:674-675; QuickGELU ``activations.py:117-123``):

  VisionTransformer: conv1 (k=s=patch, no bias) -> [CLS | patches] + pos ->
  ln_pre -> L x {x += attn(ln_1 x); x += mlp(ln_2 x)} -> ln_post(x[:,0]) @ proj
  text: tok_emb[t] + pos -> same blocks with a causal mask -> ln_final ->
  row at argmax(t) @ text_projection.

``dtype`` selects the arithmetic: float32 is the reference CPU path
(``Backend/embedding.py`` on CPU runs the fp32 model), float64
gives the high-precision truth the parity tests compare against.
"""
from __future__ import annotations

import numpy as np


def layer_norm(x, w, b, eps=1e-5):
    # OpenAI LayerNorm subclass computes in fp32 and casts back (model.py).
    mu = x.mean(-1, keepdims=True)
    xc = x - mu
    var = (xc * xc).mean(-1, keepdims=True)
    return xc / np.sqrt(var + eps) * w + b


def quick_gelu(x):
    return x * (1.0 / (1.0 + np.exp(-1.702 * x)))


def _softmax(s):
    s = s - s.max(-1, keepdims=True)
    e = np.exp(s)
    return e / e.sum(-1, keepdims=True)


def attention(x, sd, p, heads, causal):
    """nn.MultiheadAttention(d, heads) with q scaled by head_dim**-0.5."""
    B, S, W = x.shape
    dh = W // heads
    qkv = x @ sd[p + "attn.in_proj_weight"].T + sd[p + "attn.in_proj_bias"]
    q, k, v = qkv[..., :W], qkv[..., W:2 * W], qkv[..., 2 * W:]
    q = q.reshape(B, S, heads, dh).transpose(0, 2, 1, 3)
    k = k.reshape(B, S, heads, dh).transpose(0, 2, 1, 3)
    v = v.reshape(B, S, heads, dh).transpose(0, 2, 1, 3)
    s = (q @ k.transpose(0, 1, 3, 2)) * (dh ** -0.5)
    if causal:
        mask = np.triu(np.ones((S, S), dtype=bool), 1)
        s = np.where(mask, -np.inf, s)
    o = _softmax(s) @ v
    o = o.transpose(0, 2, 1, 3).reshape(B, S, W)
    return o @ sd[p + "attn.out_proj.weight"].T + sd[p + "attn.out_proj.bias"]


def resblock(x, sd, p, heads, causal):
    x = x + attention(layer_norm(x, sd[p + "ln_1.weight"], sd[p + "ln_1.bias"]), sd, p, heads, causal)
    h = layer_norm(x, sd[p + "ln_2.weight"], sd[p + "ln_2.bias"])
    h = quick_gelu(h @ sd[p + "mlp.c_fc.weight"].T + sd[p + "mlp.c_fc.bias"])
    return x + (h @ sd[p + "mlp.c_proj.weight"].T + sd[p + "mlp.c_proj.bias"])


def _cast(sd, dtype):
    return {k: np.asarray(v, dtype=dtype) for k, v in sd.items()}


def patchify(pixels, patch):
    """[B,3,R,R] -> [B, G*G, 3*P*P] with k = c*P*P + kh*P + kw (conv1 weight order)."""
    B, C, R, _ = pixels.shape
    G = R // patch
    x = pixels.reshape(B, C, G, patch, G, patch).transpose(0, 2, 4, 1, 3, 5)
    return x.reshape(B, G * G, C * patch * patch)


def encode_image(pixels, sd, cfg, dtype=np.float32, return_hidden=False):
    sd = _cast(sd, dtype)
    x = np.asarray(pixels, dtype=dtype)
    B = x.shape[0]
    W = cfg.vision_width
    wconv = sd["visual.conv1.weight"].reshape(W, -1)
    tok = patchify(x, cfg.vision_patch_size) @ wconv.T                      # conv1
    cls = np.broadcast_to(sd["visual.class_embedding"], (B, 1, W))
    x = np.concatenate([cls, tok], axis=1) + sd["visual.positional_embedding"]
    x = layer_norm(x, sd["visual.ln_pre.weight"], sd["visual.ln_pre.bias"])
    hidden = [x]
    for i in range(cfg.vision_layers):
        x = resblock(x, sd, f"visual.transformer.resblocks.{i}.", cfg.vision_heads, False)
        hidden.append(x)
    x = layer_norm(x[:, 0, :], sd["visual.ln_post.weight"], sd["visual.ln_post.bias"])
    out = x @ sd["visual.proj"]
    return (out, hidden) if return_hidden else out


def encode_text(tokens, sd, cfg, dtype=np.float32, return_hidden=False):
    sd = _cast(sd, dtype)
    tokens = np.asarray(tokens)
    x = sd["token_embedding.weight"][tokens] + sd["positional_embedding"]
    hidden = [x]
    for i in range(cfg.text_layers):
        x = resblock(x, sd, f"transformer.resblocks.{i}.", cfg.text_heads, True)
        hidden.append(x)
    x = layer_norm(x, sd["ln_final.weight"], sd["ln_final.bias"])
    eot = tokens.argmax(-1)          # EOT (49407) is the largest id in each row
    out = x[np.arange(x.shape[0]), eot] @ sd["text_projection"]
    return (out, hidden) if return_hidden else out


def cosine(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return (a * b).sum(-1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))
