"""The model object returned by ``clip.load`` — same surface as openai/CLIP's
``CLIP`` module as the reference touches it:

  model.encode_image(x)            Backend/embedding.py:49, embedding_service.py:490
  model.encode_text(tokens)        embedding_service.py:174,177, compare_models.py:1204
  model.visual.output_dim          embedding_service.py:25
  model.logit_scale                embedding_service.py:34
  model.float() / .eval() / .to()  embedding_service.py:22, :118-119 (float(): the fp32 tower, as
                                   openai/CLIP's float() makes every weight and activation fp32)
  model.state_dict() / load_state_dict()  (OpenAI keys; CLIPWithClassifier wraps them as clip_model.*)
  model(image, text)               -> (logits_per_image, logits_per_text)

Every forward runs in libmiclip's HIP kernels through the C-ABI; torch is used
only for device buffers and the current HIP stream.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from . import _native as N
from .config import CLIPConfig, from_state_dict


def _norm_code(normalize):
    """False: raw features; True: f / ||f|| (embedding_service.py:502);
    "guarded": f / ||f|| if ||f|| > 1e-8 else f (compare_models.py:1166-1171)."""
    if normalize == "guarded":
        return 2
    return int(bool(normalize))


class _Visual:
    def __init__(self, cfg: CLIPConfig):
        self.output_dim = cfg.embed_dim
        self.input_resolution = cfg.image_resolution
        self.width = cfg.vision_width
        self.layers = cfg.vision_layers
        self.patch_size = cfg.vision_patch_size


class CLIP:
    """MI355X-native CLIP (ViT image tower + causal text tower)."""

    def __init__(self, cfg: CLIPConfig, state_dict: dict, device="cuda", image_chunk=None, text_chunk=64,
                 weights: str = "bf16"):
        """``weights``:

        * "bf16" — bf16 MFMA GEMMs, fp16 vision residual stream (the throughput
          mode; the reference's own GPU path runs fp16, openai/CLIP convert_weights);
        * "fp32" — every GEMM on the exact-f32 MFMA, every activation and the
          residual stream f32 (the reference's CPU arithmetic, BASELINE.json
          configs[0]; ``model.float()`` selects it, as openai/CLIP's float() does
          for ``CLIPWithClassifier``, embedding_service.py:22) — the parity mode
          in which the R@K flow reproduces the reference's ranks (miclip.evaluate);
        * "fp8" — the vision tower's GEMMs on the block-scaled fp8 MFMA with
          MX-fp8 weights and activations (BASELINE.json configs[4])."""
        import torch

        if weights not in ("bf16", "fp8", "fp32"):
            raise N.MiClipError(f"weights must be 'bf16', 'fp32' or 'fp8', got {weights!r}")
        self.weights = weights

        self.cfg = cfg
        self._sd = {k: np.ascontiguousarray(v, dtype=np.float32) for k, v in state_dict.items()}
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise N.MiClipError("the MI355X path runs on a GPU device ('cuda' on ROCm); the CPU restatement "
                                "lives in oracle/ and is test infrastructure only")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.visual = _Visual(cfg)
        self.context_length = cfg.context_length
        self.vocab_size = cfg.vocab_size
        self.logit_scale = torch.tensor(float(np.asarray(self._sd["logit_scale"]).reshape(())))
        self._out_dtype = torch.float32
        self._lock = threading.Lock()
        if image_chunk is None:
            # ~250k token rows per pass: the GEMMs' last wave of 256x256 tiles
            # is a small fraction of the launch (at 100k rows the N = 768
            # GEMMs ran 1173 tiles = 4.6 rounds of 256 CUs); B/32 measured
            # +1.9 % at 5000-10000 frames per pass against 2000
            image_chunk = max(8, 250_000 // cfg.vision_tokens)
        self._chunks = (int(image_chunk), int(text_chunk))
        self._ctx = None
        self._build()

    # ------------------------------------------------------------------ setup
    def _build(self):
        L = N.lib()
        blob = N.pack_weights(self._sd, self.cfg)
        arch = N.Arch.from_config(self.cfg)
        ctx = ctypes.c_void_p()
        wdt = {"fp8": N.MI_FP8, "fp32": N.MI_F32}.get(self.weights, N.MI_BF16)
        N.check(L.mi_clip_create(ctypes.byref(arch), blob.ctypes.data, blob.size, self.device.index, wdt,
                                 ctypes.byref(ctx)), "mi_clip_create")
        self._ctx = ctx
        self._destroy = L.mi_clip_destroy   # the library that made the context frees it
        N.check(L.mi_clip_reserve(self._ctx, self._chunks[0], self._chunks[1]), "mi_clip_reserve")

    def close(self):
        if self._ctx is not None and self._ctx.value:
            self._destroy(self._ctx)
        self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------- module-ish API
    @property
    def dtype(self):
        return self._out_dtype

    def eval(self):
        return self

    def train(self, mode=True):
        if mode:
            raise N.MiClipError("inference-only model: training is out of scope (SURVEY.md §2.1 #16)")
        return self

    def float(self):
        """openai/CLIP ``model.float()``: weights (and so every activation) fp32.
        Here: rebuild the context on the fp32 tower (a no-op when it already is)."""
        import torch
        self._out_dtype = torch.float32
        if self.weights != "fp32":
            self.close()
            self.weights = "fp32"
            self._build()
        return self

    def half(self):
        import torch
        self._out_dtype = torch.float16
        return self

    def to(self, device=None, dtype=None):
        import torch
        if dtype is not None:
            self._out_dtype = dtype
        if device is not None:
            dev = torch.device(device)
            if dev.type == "cuda":
                dev = torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())
                if dev != self.device:
                    self.close()
                    self.device = dev
                    self._build()
            elif dev.type != "cuda":
                raise N.MiClipError("the MI355X path has no CPU execution")
        return self

    def cuda(self, device=None):
        return self.to("cuda" if device is None else f"cuda:{device}")

    def parameters(self):
        import torch
        return iter([torch.from_numpy(v) for v in self._sd.values()])

    def state_dict(self):
        import torch
        return {k: torch.from_numpy(v.copy()) for k, v in self._sd.items()}

    def load_state_dict(self, sd, strict=True):
        sd = {k: (v.detach().float().cpu().numpy() if hasattr(v, "detach") else np.asarray(v, np.float32))
              for k, v in sd.items()}
        if any(k.startswith("clip_model.") for k in sd):
            sd = {k[len("clip_model."):]: v for k, v in sd.items() if k.startswith("clip_model.")}
        cfg = from_state_dict(sd, self.cfg.name)
        if strict and set(sd) != set(self._sd):
            raise N.MiClipError("load_state_dict: key mismatch")
        self.close()
        self.cfg = cfg
        self._sd = {k: np.ascontiguousarray(v, dtype=np.float32) for k, v in sd.items()}
        self.visual = _Visual(cfg)
        self._build()
        return self

    # ---------------------------------------------------------------- forward
    def _out(self, rows, dtype=None):
        import torch
        return torch.empty((rows, self.cfg.embed_dim), dtype=dtype or self._out_dtype, device=self.device)

    def encode_image(self, image, normalize=False, out_dtype=None):
        """[B,3,R,R] pixels (normalised domain) -> [B, embed_dim]."""
        import torch
        x = image
        if not isinstance(x, torch.Tensor):
            x = torch.as_tensor(np.asarray(x))
        R = self.cfg.image_resolution
        if x.dim() != 4 or tuple(x.shape[1:]) != (3, R, R):
            raise N.MiClipError(f"encode_image expects [B,3,{R},{R}], got {tuple(x.shape)}")
        x = x.to(self.device, non_blocking=True)
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        x = x.contiguous()
        out = self._out(x.shape[0], out_dtype)
        with torch.cuda.device(self.device), self._lock:
            N.check(N.lib().mi_clip_encode_image(self._ctx, x.data_ptr(), x.shape[0], N.dtype_code(x.dtype),
                                                 out.data_ptr(), N.dtype_code(out.dtype), _norm_code(normalize),
                                                 N.stream_ptr(self.device)), "mi_clip_encode_image")
        return out

    def encode_text(self, text, normalize=False, out_dtype=None):
        """[Q, context_length] clip.tokenize ids -> [Q, embed_dim]."""
        import torch
        t = text if isinstance(text, torch.Tensor) else torch.as_tensor(np.asarray(text))
        if t.dim() != 2 or t.shape[1] != self.cfg.context_length:
            raise N.MiClipError(f"encode_text expects [Q,{self.cfg.context_length}] tokens, got {tuple(t.shape)}")
        t = t.to(device=self.device, dtype=torch.int32, non_blocking=True).contiguous()
        out = self._out(t.shape[0], out_dtype)
        with torch.cuda.device(self.device), self._lock:
            N.check(N.lib().mi_clip_encode_text(self._ctx, t.data_ptr(), t.shape[0], out.data_ptr(),
                                                N.dtype_code(out.dtype), _norm_code(normalize),
                                                N.stream_ptr(self.device)), "mi_clip_encode_text")
        return out

    def __call__(self, image, text):
        """openai/CLIP ``CLIP.forward``: (logits_per_image, logits_per_text)."""
        from .retrieval import score_matrix
        img = self.encode_image(image, out_dtype=__import__("torch").float32)
        txt = self.encode_text(text, normalize=True, out_dtype=__import__("torch").float32)
        per_text = score_matrix(img, txt, norm="l2")          # [Q, B] = t . i/|i|
        scale = float(np.exp(self.logit_scale.item()))
        logits_per_text = per_text * scale
        return logits_per_text.t().contiguous(), logits_per_text

    forward = __call__
