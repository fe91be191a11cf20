"""Weight loading policy and the no-code checkpoint readers (CPU only).

* random-init weights are opt-in (``synthetic:`` prefix, $MICLIP_SYNTHETIC_WEIGHTS,
  ``test-*`` configs); a published name without $CLIP_WEIGHTS raises, and so
  does a $CLIP_WEIGHTS file of another architecture;
* an OpenAI-style TorchScript archive is read without torch.jit.load (no code
  from the file runs) and yields exactly ``module.state_dict()``;
* a fine-tuned CLIPWithClassifier checkpoint
  (Backend/services/embedding_service.py:112-113) unwraps to ``clip_model.*``;
* ``clip.load(device="cpu")`` raises with the oracle-free policy message
  (the reference's CPU branch, Backend/embedding.py:21-22).
"""
import numpy as np
import pytest


def _tiny_sd():
    from miclip import config, weights
    return weights.make_state_dict(config.get_config("test-tiny"))


def test_resolve_policy(monkeypatch, tmp_path):
    import torch
    from miclip import _native, config, weights
    monkeypatch.delenv("CLIP_WEIGHTS", raising=False)
    monkeypatch.delenv("MICLIP_SYNTHETIC_WEIGHTS", raising=False)
    with pytest.raises(_native.MiClipError, match="no weights for ViT-B/32"):
        weights.resolve("ViT-B/32")
    cfg, sd = weights.resolve("test-tiny")                      # synthetic-only parity config
    assert cfg.name == "test-tiny" and "visual.proj" in sd
    cfg, _ = weights.resolve("synthetic:test-small")
    assert cfg.name == "test-small"
    monkeypatch.setenv("MICLIP_SYNTHETIC_WEIGHTS", "1")
    with pytest.warns(RuntimeWarning, match="random-init"):
        assert weights.resolve("ViT-B/16")[0].name == "ViT-B/16"
    # $CLIP_WEIGHTS: a checkpoint of another architecture is an error, not a silent fallback
    p = tmp_path / "small.pt"
    torch.save({k: torch.from_numpy(np.array(v)) for k, v in weights.make_state_dict(
        config.get_config("test-small")).items()}, p)
    monkeypatch.setenv("CLIP_WEIGHTS", str(p))
    with pytest.raises(_native.MiClipError, match="holds a"):
        weights.resolve("ViT-B/32")
    monkeypatch.setenv("CLIP_WEIGHTS", str(tmp_path / "missing.pt"))
    with pytest.raises(_native.MiClipError, match="not a file"):
        weights.resolve("ViT-B/32")
    cfg, sd = weights.resolve(str(p))                              # a path: its own architecture
    assert cfg.name == "test-small" and cfg.vision_width == 256


class _Block(object):
    pass


def _scripted_clip_like():
    import torch
    from torch import nn

    class Block(nn.Module):
        def __init__(self, w):
            super().__init__()
            self.ln_1 = nn.LayerNorm(w)
            self.attn = nn.MultiheadAttention(w, 2)
            self.mlp = nn.Sequential()
            self.mlp.add_module("c_fc", nn.Linear(w, 4 * w))
            self.mlp.add_module("c_proj", nn.Linear(4 * w, w))

        def forward(self, x):
            y = self.ln_1(x)
            return x + self.attn(y, y, y, need_weights=False)[0] + self.mlp.c_proj(self.mlp.c_fc(y))

    class Tower(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv1 = nn.Conv2d(3, 16, 4, 4, bias=False)
            self.class_embedding = nn.Parameter(torch.randn(16))
            self.proj = nn.Parameter(torch.randn(16, 8).half())
            self.resblocks = nn.Sequential(Block(16), Block(16))

        def forward(self, x):
            return self.resblocks(x) @ self.proj.float()

    class Model(nn.Module):
        def __init__(self):
            super().__init__()
            self.visual = Tower()
            self.positional_embedding = nn.Parameter(torch.randn(5, 16).to(torch.bfloat16))
            self.register_buffer("counter", torch.arange(6, dtype=torch.int64).reshape(2, 3).t())  # strided view

        def forward(self, x):
            return self.visual(x)

    torch.manual_seed(0)
    return torch.jit.script(Model().eval())


def test_torchscript_archive_read_without_code(tmp_path):
    import torch
    from miclip import weights
    m = _scripted_clip_like()
    p = tmp_path / "ViT-test.pt"
    m.save(str(p))
    assert weights._is_torchscript_archive(str(p))
    got = weights.read_torchscript_tensors(str(p))
    ref = m.state_dict()
    assert set(got) == set(ref)
    for k, v in ref.items():
        a = got[k]
        b = v.float().numpy() if v.dtype in (torch.bfloat16, torch.float16) else v.numpy()
        assert a.shape == b.shape, k
        np.testing.assert_array_equal(np.asarray(a, dtype=b.dtype), b, err_msg=k)
    sd = weights.load_state_dict(str(p))                           # the public loader takes the same route
    assert set(sd) == set(ref) and all(v.dtype == np.float32 for v in sd.values())


def test_refuses_code_bearing_pickle(tmp_path):
    """A plain torch.save pickle that is not weights-only is refused by the
    weights_only loader, and NOT retried with a less restricted one."""
    import pickle
    from miclip import weights
    p = tmp_path / "evil.pt"
    with open(p, "wb") as f:
        pickle.dump({"x": _Block()}, f)
    with pytest.raises(Exception) as ei:
        weights.load_state_dict(str(p))
    assert "jit" not in str(ei.value).lower()


def test_finetuned_checkpoint_unwrap(tmp_path):
    import torch
    from miclip import weights
    sd = _tiny_sd()
    msd = {f"clip_model.{k}": torch.from_numpy(np.array(v)) for k, v in sd.items()}
    msd["classifier.0.weight"] = torch.zeros(512, 128)
    msd["classifier.3.bias"] = torch.zeros(3)
    p = tmp_path / "final_checkpoint.pt"
    torch.save({"epoch": 1, "model_state_dict": msd, "optimizer_state_dict": {"state": {}, "param_groups": []},
                "loss": 0.5}, p)
    got = weights.load_state_dict(str(p))
    assert set(got) == set(sd)
    for k in sd:
        np.testing.assert_array_equal(got[k], sd[k])


def test_cpu_device_policy():
    import clip
    from miclip import _native, embedding
    with pytest.raises(_native.MiClipError, match="no CPU execution path"):
        clip.load("test-tiny", device="cpu")
    import torch
    if not torch.cuda.is_available():
        # Backend/embedding.py:21-22 picks "cpu" on a GPU-less host: the mirror says why it cannot run
        with pytest.raises(_native.MiClipError, match="oracle"):
            embedding.extract_and_save_embeddings_from_folder(".", "test-tiny")


def _ts_archive(path, size, stride, offset=0):
    """A minimal TorchScript-layout zip whose data.pkl rebuilds one tensor of
    the given geometry over a 16-float storage."""
    import collections
    import io
    import pickle
    import zipfile
    import torch

    class _Store:
        pass

    class _P(pickle.Pickler):
        def persistent_id(self, obj):
            return ("storage", torch.FloatStorage, "0", "cpu", 16) if obj is _Store else None

    class _T:
        def __reduce__(self):
            return (torch._utils._rebuild_tensor_v2, (_Store, offset, size, stride, False, collections.OrderedDict()))

    buf = io.BytesIO()
    _P(buf, protocol=2).dump({"w": _T()})
    with zipfile.ZipFile(path, "w") as zf:
        zf.writestr("m/data.pkl", buf.getvalue())
        zf.writestr("m/code/__torch__.py", "")
        zf.writestr("m/data/0", np.arange(16, dtype=np.float32).tobytes())


def test_torchscript_reader_bounds_checks_geometry(tmp_path):
    """A crafted archive must not make the reader stride outside the storage
    (as_strided has no bounds check)."""
    import pickle
    from miclip import weights
    ok = tmp_path / "ok.pt"
    _ts_archive(ok, (4, 4), (4, 1))
    np.testing.assert_array_equal(weights.read_torchscript_tensors(str(ok))["w"],
                                  np.arange(16, dtype=np.float32).reshape(4, 4))
    _ts_archive(ok, (2, 2), (1, 4), offset=10)                     # transposed view ending at element 15
    np.testing.assert_array_equal(weights.read_torchscript_tensors(str(ok))["w"], [[10, 14], [11, 15]])
    for i, (size, stride, off) in enumerate([((4, 4), (4, 1000), 0), ((4, 4), (4, 1), 1), ((2,), (1,), -1),
                                             ((3,), (-1,), 2), ((1 << 40,), (1,), 0)]):
        bad = tmp_path / f"bad{i}.pt"
        _ts_archive(bad, size, stride, off)
        with pytest.raises(pickle.UnpicklingError):
            weights.read_torchscript_tensors(str(bad))
