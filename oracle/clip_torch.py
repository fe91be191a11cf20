"""ORACLE (test infrastructure / CPU baseline only) — torch-CPU fp32
restatement of openai/CLIP inference, the form BASELINE.md's CPU-baseline plan
times: ``Backend/embedding.py`` on a CPU host runs openai/CLIP's fp32 model
(``clip.load(..., device="cpu")`` keeps fp32, embedding.py:21-22) one image
per call (embedding.py:39-52).  Same graph as ``clip_ref`` (the numpy
restatement, checked equal in tests/test_oracle.py): conv1 as a strided
Conv2d, [CLS | patches] + pos, ln_pre, pre-LN blocks with
nn.MultiheadAttention semantics, QuickGELU, ln_post on CLS, ``@ proj``; the
text tower with the causal mask and argmax (EOT) pooling.

Never imported by the product; ``bench.py`` uses it only in its
``cpu_baseline`` leg, outside the timed GPU region.
"""
from __future__ import annotations

import numpy as np


class TorchCLIP:
    def __init__(self, sd, cfg):
        import torch
        self.cfg = cfg
        self.t = {k: torch.from_numpy(np.ascontiguousarray(np.asarray(v, dtype=np.float32))) for k, v in sd.items()}

    def _block(self, x, p, heads, causal):
        import torch
        import torch.nn.functional as F
        t = self.t
        B, S, W = x.shape
        dh = W // heads
        h = F.layer_norm(x, (W,), t[p + "ln_1.weight"], t[p + "ln_1.bias"], 1e-5)
        qkv = F.linear(h, t[p + "attn.in_proj_weight"], t[p + "attn.in_proj_bias"])
        q, k, v = qkv.split(W, dim=-1)
        q = q.reshape(B, S, heads, dh).transpose(1, 2)
        k = k.reshape(B, S, heads, dh).transpose(1, 2)
        v = v.reshape(B, S, heads, dh).transpose(1, 2)
        s = (q * dh ** -0.5) @ k.transpose(-1, -2)
        if causal:
            s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool), 1), float("-inf"))
        o = (s.softmax(-1) @ v).transpose(1, 2).reshape(B, S, W)
        x = x + F.linear(o, t[p + "attn.out_proj.weight"], t[p + "attn.out_proj.bias"])
        h = F.layer_norm(x, (W,), t[p + "ln_2.weight"], t[p + "ln_2.bias"], 1e-5)
        h = F.linear(h, t[p + "mlp.c_fc.weight"], t[p + "mlp.c_fc.bias"])
        h = h * torch.sigmoid(1.702 * h)
        return x + F.linear(h, t[p + "mlp.c_proj.weight"], t[p + "mlp.c_proj.bias"])

    def encode_image(self, pixels):
        import torch
        import torch.nn.functional as F
        cfg, t = self.cfg, self.t
        with torch.no_grad():
            x = torch.as_tensor(pixels, dtype=torch.float32)
            B = x.shape[0]
            W = cfg.vision_width
            x = F.conv2d(x, t["visual.conv1.weight"], stride=cfg.vision_patch_size)      # [B, W, G, G]
            x = x.reshape(B, W, -1).transpose(1, 2)
            x = torch.cat([t["visual.class_embedding"].expand(B, 1, W), x], dim=1) + t["visual.positional_embedding"]
            x = F.layer_norm(x, (W,), t["visual.ln_pre.weight"], t["visual.ln_pre.bias"], 1e-5)
            for i in range(cfg.vision_layers):
                x = self._block(x, f"visual.transformer.resblocks.{i}.", cfg.vision_heads, False)
            x = F.layer_norm(x[:, 0], (W,), t["visual.ln_post.weight"], t["visual.ln_post.bias"], 1e-5)
            return (x @ t["visual.proj"]).numpy()

    def encode_text(self, tokens):
        import torch
        import torch.nn.functional as F
        cfg, t = self.cfg, self.t
        with torch.no_grad():
            tk = torch.as_tensor(np.asarray(tokens), dtype=torch.int64)
            x = t["token_embedding.weight"][tk] + t["positional_embedding"]
            for i in range(cfg.text_layers):
                x = self._block(x, f"transformer.resblocks.{i}.", cfg.text_heads, True)
            x = F.layer_norm(x, (cfg.text_width,), t["ln_final.weight"], t["ln_final.bias"], 1e-5)
            x = x[torch.arange(x.shape[0]), tk.argmax(-1)]
            return (x @ t["text_projection"]).numpy()
