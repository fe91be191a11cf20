"""ctypes binding of ``libmiclip.so`` (C-ABI declared in ``include/miclip.h``).

There is deliberately no CPU fallback: if the library is missing or cannot be
loaded, every entry point raises.  ``torch`` is used only for device memory,
streams and dtypes (plumbing); all compute runs in the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .config import CLIPConfig

LIB_NAME = "libmiclip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# the sources both libraries are built from (their fingerprint is checked at load, _check_sources)
CSRC_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
# the A/B build (csrc `make ab`): the same C-ABI plus every alternative kernel
# schedule, ablation and probe; used by scripts/*_micro.py (MICLIP_LIB=ab) and
# the bit-identity tests of the alternatives, never by the product path
AB_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                           "scripts", "ab", "libmiclip_ab.so")

MI_F32, MI_BF16, MI_F16, MI_FP8 = 0, 1, 2, 3
MI_NAN_FIRST, MI_NAN_LAST = 0, 1
MI_NORM_L2, MI_NORM_L2_GUARD, MI_NORM_NONE = 0, 1, 2
MI_PREP_CLIP, MI_PREP_SQUASH = 0, 1
MI_RESAMPLE_BICUBIC, MI_RESAMPLE_BILINEAR = 0, 1

# every symbol include/miclip.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "mi_abi_version", "mi_build_id", "mi_build_sources", "mi_last_error", "mi_clip_weights_numel", "mi_clip_create", "mi_clip_destroy",
    "mi_clip_reserve", "mi_clip_encode_image", "mi_clip_encode_text", "mi_rank_workspace_bytes",
    "mi_rank_topk", "mi_rank_merge", "mi_score_matrix", "mi_rank_of_targets",
    "mi_op_gemm", "mi_op_gemm_f32", "mi_op_layernorm", "mi_op_attention", "mi_op_residual_ln",
    "mi_op_residual_stats", "mi_op_gemm_ln", "mi_op_gemm_residual", "mi_op_split6",
    "mi_resample_coeffs", "mi_preprocess_workspace_bytes", "mi_preprocess_frames",
    "mi_jpeg_workspace_bytes", "mi_jpeg_decode", "mi_host_gather",
    "mi_op_quantize_mx", "mi_op_gemm_mx",
    "mi_mirror_build", "mi_rank_mirror_workspace_bytes", "mi_rank_mirror", "mi_normalize_rows_f16",
    "mi_jpeg_decode_transform", "mi_op_split2h", "mi_op_gemm_split2h", "mi_op_attention_f32",
    "mi_op_attention_f32_split",
    "mi_clip_kernel_events", "mi_clip_kernel_times",
)


class MiClipError(RuntimeError):
    pass


class Arch(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "embed_dim", "image_resolution", "vision_layers", "vision_width", "vision_patch_size",
        "context_length", "vocab_size", "text_width", "text_heads", "text_layers")]

    @classmethod
    def from_config(cls, cfg: CLIPConfig) -> "Arch":
        return cls(cfg.embed_dim, cfg.image_resolution, cfg.vision_layers, cfg.vision_width,
                   cfg.vision_patch_size, cfg.context_length, cfg.vocab_size, cfg.text_width,
                   cfg.text_heads, cfg.text_layers)


_lib = None
_lib_ab = None


def lib():
    """Load libmiclip.so once; raise if it is absent (no silent fallback).
    ``$MICLIP_LIB=ab`` loads the A/B build instead (measurement scripts)."""
    global _lib
    if _lib is not None:
        return _lib
    if os.environ.get("MICLIP_LIB") == "ab":
        _lib = lib_ab()
        return _lib
    if not os.path.isfile(LIB_PATH):
        raise MiClipError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                          " or `make -C <pkg>/csrc`")
    _lib = _bind(LIB_PATH)
    return _lib


def lib_ab():
    """The A/B library (scripts/ab/libmiclip_ab.so); raises if it is not built."""
    global _lib_ab
    if _lib_ab is not None:
        return _lib_ab
    if not os.path.isfile(AB_LIB_PATH):
        raise MiClipError(f"{AB_LIB_PATH} not found: `make -C <pkg>/csrc ab`")
    _lib_ab = _bind(AB_LIB_PATH)
    return _lib_ab


def _bind(path):
    # torch ships its own libamdhip64 with the same SONAME (libamdhip64.so.7)
    # as /opt/rocm's.  Loading torch first makes the dynamic linker bind
    # libmiclip to torch's HIP runtime, so tensors, streams and our kernels
    # live in ONE runtime; the other order makes torch bind to /opt/rocm's
    # runtime and fail ("No HIP GPUs are available").
    import torch  # noqa: F401
    L = ctypes.CDLL(path)
    P, I32, I64, SZ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
    sig = {
        "mi_abi_version": (ctypes.c_int, []),
        "mi_build_id": (ctypes.c_char_p, []),
        "mi_build_sources": (ctypes.c_char_p, []),
        "mi_last_error": (ctypes.c_char_p, []),
        "mi_clip_weights_numel": (I64, [ctypes.POINTER(Arch)]),
        "mi_clip_create": (ctypes.c_int, [ctypes.POINTER(Arch), P, I64, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(P)]),
        "mi_clip_destroy": (ctypes.c_int, [P]),
        "mi_clip_reserve": (ctypes.c_int, [P, I64, I64]),
        "mi_clip_encode_image": (ctypes.c_int, [P, P, I64, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P]),
        "mi_clip_encode_text": (ctypes.c_int, [P, P, I64, P, ctypes.c_int, ctypes.c_int, P]),
        "mi_rank_workspace_bytes": (SZ, [I64, I64, I32]),
        "mi_rank_topk": (ctypes.c_int, [P, I64, I64, ctypes.c_int, P, I64, I32, I64, ctypes.c_int, ctypes.c_int,
                                        P, P, P, SZ, P]),
        "mi_rank_merge": (ctypes.c_int, [P, P, I64, I64, I32, ctypes.c_int, P, P, P]),
        "mi_mirror_build": (ctypes.c_int, [P, I64, I64, ctypes.c_int, P, P]),
        "mi_rank_mirror_workspace_bytes": (SZ, [I64, I64]),
        "mi_normalize_rows_f16": (ctypes.c_int, [P, I64, I64, P, P]),
        "mi_rank_mirror": (ctypes.c_int, [P, P, I64, I64, ctypes.c_int, P, I64, I32, I64, ctypes.c_int, P, P, P, P,
                                          SZ, P]),
        "mi_score_matrix": (ctypes.c_int, [P, I64, I64, ctypes.c_int, P, I64, ctypes.c_int, P, P]),
        "mi_rank_of_targets": (ctypes.c_int, [P, I64, I64, P, P, I64, P, P]),
        "mi_op_gemm": (ctypes.c_int, [P, P, P, P, I32, I32, I32, I32, P]),
        "mi_op_gemm_f32": (ctypes.c_int, [P, P, P, P, I32, I32, I32, I32, P]),
        "mi_op_layernorm": (ctypes.c_int, [P, P, P, P, I32, I32, P]),
        "mi_op_attention": (ctypes.c_int, [P, P, I32, I32, I32, I32, P]),
        "mi_op_residual_ln": (ctypes.c_int, [P, P, P, P, P, I32, I32, I32, P]),
        "mi_op_residual_stats": (ctypes.c_int, [P, P, P, I32, I32, P]),
        "mi_op_gemm_ln": (ctypes.c_int, [P, I64, P, P, P, P, P, I32, I32, I32, I32, P]),
        "mi_op_gemm_residual": (ctypes.c_int, [P, I64, P, I64, P, P, P, P, I32, I32, I32, P]),
        "mi_op_split6": (ctypes.c_int, [P, I64, I64, I32, I32, I32, P, P]),
        "mi_op_split2h": (ctypes.c_int, [P, I64, I64, I32, I32, I32, P, P, P]),
        "mi_op_gemm_split2h": (ctypes.c_int, [P, P, P, P, P, P, I32, I32, I32, I32, P]),
        "mi_op_attention_f32": (ctypes.c_int, [P, P, I32, I32, I32, I32, P]),
        "mi_op_attention_f32_split": (ctypes.c_int, [P, P, ctypes.c_float, ctypes.c_float, P, I32, P, I32, I32, I32, I32,
                                                     P]),
        "mi_clip_kernel_events": (ctypes.c_int, [P, I32, I32]),
        "mi_clip_kernel_times": (ctypes.c_int, [P, P, I32]),
        "mi_op_quantize_mx": (ctypes.c_int, [P, P, P, I32, I32, P]),
        "mi_op_gemm_mx": (ctypes.c_int, [P, P, P, P, P, P, I32, I32, I32, I32, P]),
        "mi_resample_coeffs": (ctypes.c_int, [I32, ctypes.c_double, ctypes.c_double, I32, ctypes.c_int, P, I64, P]),
        "mi_preprocess_workspace_bytes": (SZ, [I64, I32, I32, I32, ctypes.c_int]),
        "mi_preprocess_frames": (ctypes.c_int, [P, I64, I32, I32, I32, ctypes.c_int, P, ctypes.c_int, P, SZ, P]),
        "mi_jpeg_workspace_bytes": (SZ, [P, I32, I64]),
        "mi_jpeg_decode": (ctypes.c_int, [P, I64, P, P, P, P, I32, P, P, I32, P, P, SZ, P]),
        "mi_jpeg_decode_transform": (ctypes.c_int, [P, I64, P, P, P, P, I32, P, P, I32, I32, ctypes.c_int, P,
                                                    ctypes.c_int, P, SZ, P]),
        "mi_host_gather": (ctypes.c_int, [P, P, P, I64, I32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.mi_abi_version() != 7:
        raise MiClipError("libmiclip ABI version mismatch")
    _check_sources(L, path)
    return L


def source_fingerprint(names, csrc=None):
    """The Makefile's fingerprint of `names` (paths relative to csrc/): the first 16 hex digits of
    the sha256 of the files concatenated in that order (``cat ... | sha256sum``)."""
    import hashlib
    csrc = csrc or CSRC_DIR
    h = hashlib.sha256()
    for n in names:
        with open(os.path.join(csrc, n), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _check_sources(L, path):
    """Refuse a library built from other sources than the csrc/ next to it (a stale or foreign
    binary): its mi_build_id must equal the fingerprint of the files it names.  A library shipped
    without its sources is not checked."""
    if not os.path.isdir(CSRC_DIR):
        return
    names = L.mi_build_sources().decode().split()
    missing = [n for n in names if not os.path.isfile(os.path.join(CSRC_DIR, n))]
    if missing:
        raise MiClipError(f"{path}: built from sources missing here ({', '.join(missing)}); rebuild with build()")
    built, here = L.mi_build_id().decode(), source_fingerprint(names)
    if built != here:
        raise MiClipError(f"{path} was built from other sources (fingerprint {built}) than {CSRC_DIR} ({here}): "
                          "rebuild with `python -c 'import __graft_entry__ as g; g.build()'` or `make -C <pkg>/csrc`")


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().mi_last_error().decode(errors="replace")
        raise MiClipError(f"{what} failed ({rc}): {msg}")


def weight_order(cfg: CLIPConfig):
    """Canonical blob order (DESIGN.md "Weight blob"): OpenAI state-dict keys."""
    def tower(prefix, layers):
        keys = []
        for i in range(layers):
            p = f"{prefix}resblocks.{i}."
            keys += [p + k for k in ("ln_1.weight", "ln_1.bias", "attn.in_proj_weight", "attn.in_proj_bias",
                                     "attn.out_proj.weight", "attn.out_proj.bias", "ln_2.weight", "ln_2.bias",
                                     "mlp.c_fc.weight", "mlp.c_fc.bias", "mlp.c_proj.weight", "mlp.c_proj.bias")]
        return keys
    return (["visual.conv1.weight", "visual.class_embedding", "visual.positional_embedding",
             "visual.ln_pre.weight", "visual.ln_pre.bias"] + tower("visual.transformer.", cfg.vision_layers)
            + ["visual.ln_post.weight", "visual.ln_post.bias", "visual.proj",
               "token_embedding.weight", "positional_embedding"] + tower("transformer.", cfg.text_layers)
            + ["ln_final.weight", "ln_final.bias", "text_projection", "logit_scale"])


def pack_weights(sd, cfg: CLIPConfig) -> np.ndarray:
    parts = []
    for k in weight_order(cfg):
        if k not in sd:
            raise MiClipError(f"state dict is missing {k}")
        parts.append(np.ascontiguousarray(np.asarray(sd[k], dtype=np.float32)).reshape(-1))
    blob = np.concatenate(parts)
    expect = lib().mi_clip_weights_numel(ctypes.byref(Arch.from_config(cfg)))
    if blob.size != expect:
        raise MiClipError(f"packed {blob.size} weights, the library expects {expect}")
    return blob


def stream_ptr(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(t) -> int:
    import torch
    m = {torch.float32: MI_F32, torch.bfloat16: MI_BF16, torch.float16: MI_F16}
    if t not in m:
        raise MiClipError(f"unsupported dtype {t}")
    return m[t]
