"""Portable deterministic weights and synthetic inputs.

There are no CLIP checkpoints offline, so parity and
benchmarks run on random-init weights of the real architecture, produced by a
counter-based generator that gives bit-identical float32 tensors on any host:
splitmix64 of (seed, crc32(name), element index) -> four 16-bit uniforms ->
Irwin-Hall(4) approximate normal.  Every step is exact integer arithmetic or a
single correctly-rounded IEEE operation, so the GPU box regenerates exactly the
tensors the golden fixtures were computed from.

The parameter layout is the OpenAI state dict consumed by ``clip.load``
(openai/CLIP ``model.py``; call sites ``Backend/embedding.py:22``,
``Backend/services/embedding_service.py:86``), and the standard deviations
follow openai/CLIP ``CLIP.initialize_parameters`` (text tower) and the PyTorch
defaults it leaves in place (vision tower).  LayerNorm gains/biases and linear
biases are perturbed away from 1/0 so that a swapped or dropped parameter
shows up in the parity tests.
"""
from __future__ import annotations

import os
import zlib

import numpy as np

from .config import CLIPConfig, from_state_dict

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_SQRT3 = float(np.sqrt(np.float64(3.0)))

WEIGHT_SEED = 2
PIXEL_SEED = 0
TOKEN_SEED = 1
CORPUS_SEED = 3

SOT_TOKEN = 49406
EOT_TOKEN = 49407


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = x + np.uint64(0x9E3779B97F4A7C15)
    z = x
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _stream_key(seed: int, name: str) -> np.uint64:
    return np.uint64(((seed & 0xFFFFFFFF) << 32) | (zlib.crc32(name.encode()) & 0xFFFFFFFF))


def hash_u64(seed: int, name: str, n: int, offset: int = 0) -> np.ndarray:
    key = _splitmix64(np.array([_stream_key(seed, name)], dtype=np.uint64))[0]
    idx = np.arange(offset, offset + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return _splitmix64(idx * np.uint64(0xD1B54A32D192ED03) ^ key)


def normal(seed: int, name: str, shape, std: float = 1.0, mean: float = 0.0,
           chunk: int = 1 << 22) -> np.ndarray:
    """Deterministic approximately-N(mean, std^2) float32 tensor."""
    n = int(np.prod(shape)) if len(shape) else 1
    out = np.empty(n, dtype=np.float32)
    with np.errstate(over="ignore"):
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            h = hash_u64(seed, name, e - s, s)
            acc = np.zeros(e - s, dtype=np.float64)
            for j in range(4):
                u = ((h >> np.uint64(16 * j)) & np.uint64(0xFFFF)).astype(np.float64)
                acc += u
            # each u/65536 + 0.5/65536 ~ U(0,1): sum of four has mean 2, var 1/3
            z = (acc + 2.0) / 65536.0 - 2.0
            out[s:e] = (z * (_SQRT3 * std) + mean).astype(np.float32)
    return out.reshape(shape)


def uniform_int(seed: int, name: str, shape, lo: int, hi: int) -> np.ndarray:
    """Deterministic integers in [lo, hi)."""
    n = int(np.prod(shape))
    h = hash_u64(seed, name, n)
    return (lo + (h % np.uint64(hi - lo)).astype(np.int64)).reshape(shape)


def make_state_dict(cfg: CLIPConfig, seed: int = WEIGHT_SEED) -> dict:
    """OpenAI-layout float32 state dict (numpy arrays) for ``cfg``."""
    sd = {}
    g = lambda name, shape, std, mean=0.0: normal(seed, name, shape, std, mean)  # noqa: E731

    def tower(prefix, width, layers):
        attn_std = width ** -0.5
        proj_std = (width ** -0.5) * ((2 * layers) ** -0.5)
        fc_std = (2 * width) ** -0.5
        for i in range(layers):
            p = f"{prefix}resblocks.{i}."
            sd[p + "attn.in_proj_weight"] = g(p + "attn.in_proj_weight", (3 * width, width), attn_std)
            sd[p + "attn.in_proj_bias"] = g(p + "attn.in_proj_bias", (3 * width,), 0.02)
            sd[p + "attn.out_proj.weight"] = g(p + "attn.out_proj.weight", (width, width), proj_std)
            sd[p + "attn.out_proj.bias"] = g(p + "attn.out_proj.bias", (width,), 0.02)
            sd[p + "ln_1.weight"] = g(p + "ln_1.weight", (width,), 0.1, 1.0)
            sd[p + "ln_1.bias"] = g(p + "ln_1.bias", (width,), 0.02)
            sd[p + "mlp.c_fc.weight"] = g(p + "mlp.c_fc.weight", (4 * width, width), fc_std)
            sd[p + "mlp.c_fc.bias"] = g(p + "mlp.c_fc.bias", (4 * width,), 0.02)
            sd[p + "mlp.c_proj.weight"] = g(p + "mlp.c_proj.weight", (width, 4 * width), proj_std)
            sd[p + "mlp.c_proj.bias"] = g(p + "mlp.c_proj.bias", (width,), 0.02)
            sd[p + "ln_2.weight"] = g(p + "ln_2.weight", (width,), 0.1, 1.0)
            sd[p + "ln_2.bias"] = g(p + "ln_2.bias", (width,), 0.02)

    W = cfg.vision_width
    scale = W ** -0.5
    P = cfg.vision_patch_size
    fan_in = 3 * P * P
    sd["visual.class_embedding"] = g("visual.class_embedding", (W,), scale)
    sd["visual.positional_embedding"] = g("visual.positional_embedding", (cfg.vision_tokens, W), scale)
    sd["visual.proj"] = g("visual.proj", (W, cfg.embed_dim), scale)
    sd["visual.conv1.weight"] = g("visual.conv1.weight", (W, 3, P, P), (1.0 / fan_in) ** 0.5)
    sd["visual.ln_pre.weight"] = g("visual.ln_pre.weight", (W,), 0.1, 1.0)
    sd["visual.ln_pre.bias"] = g("visual.ln_pre.bias", (W,), 0.02)
    sd["visual.ln_post.weight"] = g("visual.ln_post.weight", (W,), 0.1, 1.0)
    sd["visual.ln_post.bias"] = g("visual.ln_post.bias", (W,), 0.02)
    tower("visual.transformer.", W, cfg.vision_layers)

    TW = cfg.text_width
    sd["token_embedding.weight"] = g("token_embedding.weight", (cfg.vocab_size, TW), 0.02)
    sd["positional_embedding"] = g("positional_embedding", (cfg.context_length, TW), 0.01)
    sd["ln_final.weight"] = g("ln_final.weight", (TW,), 0.1, 1.0)
    sd["ln_final.bias"] = g("ln_final.bias", (TW,), 0.02)
    sd["text_projection"] = g("text_projection", (TW, cfg.embed_dim), TW ** -0.5)
    sd["logit_scale"] = np.array(np.log(1 / 0.07), dtype=np.float32)
    tower("transformer.", TW, cfg.text_layers)
    return sd


def synthetic_pixels(n: int, resolution: int, seed: int = PIXEL_SEED, offset: int = 0) -> np.ndarray:
    """[n,3,R,R] float32 frames already in the normalised domain."""
    per = 3 * resolution * resolution
    out = np.empty((n, per), dtype=np.float32)
    for i in range(n):
        out[i] = normal(seed, f"pixels.{offset + i}", (per,))
    return out.reshape(n, 3, resolution, resolution)


def synthetic_tokens(q: int, context_length: int = 77, vocab_size: int = 49408,
                     seed: int = TOKEN_SEED, offset: int = 0) -> np.ndarray:
    """[q,77] int32 rows ``[SOT] + L ids in [256, EOT) + [EOT]`` zero padded, L in [5,30]
    (SURVEY.md §8(d)).  For a vocab smaller than CLIP's, SOT/EOT are the two
    largest ids so that EOT stays the row argmax (the pooling rule)."""
    sot, eot = (SOT_TOKEN, EOT_TOKEN) if vocab_size == 49408 else (vocab_size - 2, vocab_size - 1)
    lo = 256 if vocab_size == 49408 else 1
    out = np.zeros((q, context_length), dtype=np.int32)
    for r in range(q):
        L = int(uniform_int(seed, f"toklen.{offset + r}", (1,), 5, 31)[0])
        L = min(L, context_length - 2)
        ids = uniform_int(seed, f"tokids.{offset + r}", (L,), lo, sot)
        out[r, 0] = sot
        out[r, 1:1 + L] = ids
        out[r, 1 + L] = eot
    return out


def synthetic_corpus(n: int, d: int, seed: int = CORPUS_SEED) -> np.ndarray:
    """[n,d] float32 L2-normalised rows (ranking microbench corpus)."""
    x = normal(seed, "corpus", (n, d))
    return x / np.linalg.norm(x, axis=-1, keepdims=True)


_STORAGE_DTYPES = {
    "FloatStorage": np.float32, "HalfStorage": np.float16, "DoubleStorage": np.float64,
    "BFloat16Storage": "bf16", "LongStorage": np.int64, "IntStorage": np.int32, "ShortStorage": np.int16,
    "CharStorage": np.int8, "ByteStorage": np.uint8, "BoolStorage": np.bool_,
}


def _is_torchscript_archive(path: str) -> bool:
    import zipfile
    if not zipfile.is_zipfile(path):
        return False
    with zipfile.ZipFile(path) as zf:
        return any(n.split("/", 1)[-1].startswith("code/") for n in zf.namelist())


def read_torchscript_tensors(path: str) -> dict:
    """Tensors of a TorchScript archive (openai/CLIP's ``ViT-B-32.pt`` form)
    WITHOUT executing anything from the file.

    The archive's ``data.pkl`` describes the module tree; it is read by a
    restricted unpickler that resolves only tensor-rebuild functions, storage
    type markers and ``OrderedDict``; every ``__torch__.*`` module class becomes
    an inert record of its attribute dict.  No TorchScript code is loaded or run
    (``torch.jit.load`` would compile and run the archive's ``code/``).  The
    attribute paths of the tensors are the OpenAI state-dict keys, as
    ``model.state_dict()`` after ``torch.jit.load`` would name them (openai/CLIP
    ``clip.load(jit=False)`` builds its model from exactly that dict)."""
    import collections
    import io
    import pickle
    import zipfile

    class _Module:                       # inert stand-in for a __torch__.* class
        def __init__(self, *a, **k):
            self._state = {}

        def __setstate__(self, state):
            self._state = state if isinstance(state, dict) else {"__state__": state}

    class _StorageType:
        def __init__(self, name):
            self.name = name

    def rebuild_tensor(storage, offset, size, stride, *rest):
        # as_strided does no bounds checking: a crafted offset / size / stride must not read
        # outside the storage buffer, so the extent is checked first
        base = storage
        size, stride = tuple(size), tuple(stride)
        if not isinstance(offset, int) or offset < 0 or len(size) != len(stride) or \
                any(not isinstance(v, int) or v < 0 for v in size + stride):
            raise pickle.UnpicklingError(f"bad tensor geometry: offset {offset}, size {size}, stride {stride}")
        numel = int(np.prod(size, dtype=np.int64)) if size else 1
        if numel > 0:
            last = offset + sum((n - 1) * st for n, st in zip(size, stride))
            if last >= len(base):
                raise pickle.UnpicklingError(f"tensor extends past its storage ({last} >= {len(base)})")
        elif offset > len(base):
            raise pickle.UnpicklingError(f"tensor offset {offset} past its storage ({len(base)})")
        return np.lib.stride_tricks.as_strided(
            base[offset:], shape=size, strides=tuple(st * base.itemsize for st in stride)).copy()

    def rebuild_parameter(data, *rest):
        return data

    with zipfile.ZipFile(path) as zf:
        names = zf.namelist()
        pkl = next(n for n in names if n.endswith("/data.pkl") or n == "data.pkl")
        root = pkl[: -len("data.pkl")]
        storages = {}

        def storage(key, typ):
            if key not in storages:
                raw = zf.read(f"{root}data/{key}")
                dt = _STORAGE_DTYPES.get(typ.name if isinstance(typ, _StorageType) else str(typ))
                if dt is None:
                    raise pickle.UnpicklingError(f"unsupported storage type {typ}")
                if dt == "bf16":
                    u = np.frombuffer(raw, dtype=np.uint16).astype(np.uint32) << np.uint32(16)
                    storages[key] = u.view(np.float32)
                else:
                    storages[key] = np.frombuffer(raw, dtype=dt)
            return storages[key]

        class _Restricted(pickle.Unpickler):
            def find_class(self, module, name):
                if module == "torch._utils" and name in ("_rebuild_tensor_v2", "_rebuild_tensor"):
                    return rebuild_tensor
                if module == "torch._utils" and name == "_rebuild_parameter":
                    return rebuild_parameter
                if module == "collections" and name == "OrderedDict":
                    return collections.OrderedDict
                if module == "torch" and name.endswith("Storage"):
                    return _StorageType(name)
                if module == "torch.jit._pickle":          # TorchScript's typed-list markers: plain data
                    if name in ("build_intlist", "build_doublelist", "build_boollist", "build_tensorlist",
                                "build_complexlist"):
                        return list
                    if name == "restore_type_tag":
                        return lambda value, type_str: value
                if module.startswith("__torch__"):
                    return type(name, (_Module,), {})
                raise pickle.UnpicklingError(f"refusing to resolve {module}.{name} from a TorchScript archive")

            def persistent_load(self, pid):
                # ('storage', storage_type, key, location, numel)
                if not (isinstance(pid, tuple) and pid and pid[0] == "storage"):
                    raise pickle.UnpicklingError(f"unexpected persistent id {pid!r}")
                return storage(str(pid[2]), pid[1])

        obj = _Restricted(io.BytesIO(zf.read(pkl))).load()

    out = {}

    def walk(o, prefix):
        if isinstance(o, np.ndarray):
            out[prefix[:-1]] = o
        elif isinstance(o, _Module):
            for k, v in o._state.items():
                walk(v, f"{prefix}{k}.")
        elif isinstance(o, dict):
            for k, v in o.items():
                walk(v, f"{prefix}{k}.")

    walk(obj, "")
    return out


def load_state_dict(path: str) -> dict:
    """Load an OpenAI-layout state dict from a LOCAL file (``$CLIP_WEIGHTS``).

    Accepted: ``.safetensors``, a plain ``torch.save`` state dict
    (``weights_only=True``), or an OpenAI TorchScript archive (its tensors are
    read by ``read_torchscript_tensors``, which executes nothing from the file).
    A fine-tuned ``CLIPWithClassifier`` checkpoint
    (``{'model_state_dict': {'clip_model.*', 'classifier.*'}}``,
    ``Backend/services/embedding_service.py:112-113``) is unwrapped to its
    ``clip_model.*`` part.  Any other file is refused with the loader's own
    error (no second, less restricted deserializer is tried)."""
    sd = _read_tensors(path)
    if any(k.startswith("clip_model.") for k in sd):
        sd = {k[len("clip_model."):]: v for k, v in sd.items() if k.startswith("clip_model.")}
    for k in ("input_resolution", "context_length", "vocab_size"):
        sd.pop(k, None)
    return {k: np.ascontiguousarray(v, dtype=np.float32) for k, v in sd.items()}


def load_classifier(path: str):
    """The ``classifier.*`` head of a fine-tuned ``CLIPWithClassifier`` checkpoint
    (nn.Sequential(Linear(D, 512), ReLU, Dropout, Linear(512, 3)):
    ``{'0.weight', '0.bias', '3.weight', '3.bias'}``, embedding_service.py:26-31),
    or None when the file has none.  Same loaders as ``load_state_dict``."""
    sd = _read_tensors(path)
    head = {k[len("classifier."):]: np.ascontiguousarray(v, dtype=np.float32) for k, v in sd.items()
            if k.startswith("classifier.")}
    return head or None


def _read_tensors(path: str) -> dict:
    import torch

    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        sd = load_file(path)
    elif _is_torchscript_archive(path):
        sd = read_torchscript_tensors(path)
    else:
        obj = torch.load(path, map_location="cpu", weights_only=True)
        if isinstance(obj, dict) and "model_state_dict" in obj:
            obj = obj["model_state_dict"]
        if not isinstance(obj, dict):
            raise RuntimeError(f"{path}: expected a state dict, got {type(obj).__name__}")
        sd = {k: (v.float().numpy() if hasattr(v, "numpy") else np.asarray(v)) for k, v in obj.items()}
    return sd


SYNTHETIC_ENV = "MICLIP_SYNTHETIC_WEIGHTS"
SYNTHETIC_PREFIX = "synthetic:"


def resolve(name_or_path: str):
    """(cfg, state_dict) for a model name or a local checkpoint path.

    * a path to a local checkpoint: its weights (architecture inferred);
    * a published name ("ViT-B/32", ...): the weights of the LOCAL file
      ``$CLIP_WEIGHTS`` (there is no download); a file of another
      architecture is an error;
    * deterministic random-init weights of the architecture only when asked
      for: the ``synthetic:`` name prefix, ``$MICLIP_SYNTHETIC_WEIGHTS=1``
      (tests, bench), or the ``test-*`` parity configurations, which exist only
      with synthetic weights.  Otherwise loading raises, so the drop-in never
      ranks frames with a meaningless model by accident."""
    import warnings
    from ._native import MiClipError
    from .config import get_config

    if os.path.isfile(name_or_path):
        sd = load_state_dict(name_or_path)
        return from_state_dict(sd), sd
    synthetic = name_or_path.startswith(SYNTHETIC_PREFIX)
    name = name_or_path[len(SYNTHETIC_PREFIX):] if synthetic else name_or_path
    cfg = get_config(name)
    test_cfg = cfg.name.startswith("test-")
    env = os.environ.get("CLIP_WEIGHTS")
    if env and not synthetic and not test_cfg:
        if not os.path.isfile(env):
            raise MiClipError(f"$CLIP_WEIGHTS={env!r} is not a file")
        sd = load_state_dict(env)
        real = from_state_dict(sd)
        if real.name != cfg.name:
            raise MiClipError(f"$CLIP_WEIGHTS={env!r} holds a {real.name} checkpoint, but {cfg.name} was requested")
        return real, sd
    if synthetic or test_cfg or os.environ.get(SYNTHETIC_ENV) == "1":
        if not test_cfg and not synthetic:
            warnings.warn(f"{cfg.name}: deterministic random-init weights (${SYNTHETIC_ENV}=1); embeddings and "
                          f"rankings are meaningless outside tests and benchmarks", RuntimeWarning, stacklevel=3)
        return cfg, make_state_dict(cfg)
    raise MiClipError(f"no weights for {cfg.name}: set $CLIP_WEIGHTS to a local OpenAI checkpoint "
                      f"(.pt TorchScript archive, state-dict .pt or .safetensors) or pass its path to clip.load; "
                      f"random-init weights need '{SYNTHETIC_PREFIX}{cfg.name}' or ${SYNTHETIC_ENV}=1")
