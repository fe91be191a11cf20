"""CPU: libmiclip.so loads, exports every symbol include/miclip.h declares, and
validates arguments before touching a GPU (no compute calls here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, state_dict


def _declared():
    hdr = open(os.path.join(ROOT, "include", "miclip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(mi_[a-z_0-9]+)\s*\(", hdr, re.M)))


def test_header_and_binding_agree():
    from miclip import _native
    assert _declared() == sorted(_native.EXPORTS)


def test_library_exports_every_symbol():
    from miclip import _native
    L = _native.lib()
    for name in _declared():
        assert hasattr(L, name), name
    out = os.popen(f"nm -D --defined-only {_native.LIB_PATH}").read()
    for name in _declared():
        assert re.search(rf"\bT {name}$", out, re.M), f"{name} not exported"
    assert L.mi_abi_version() == 7


def test_library_fingerprint_matches_its_sources(tmp_path):
    """Both libraries carry the fingerprint of the sources they were built from
    (mi_build_id: sha256 of the files mi_build_sources names); the loader recomputes it from
    csrc/ and refuses a mismatch, so a stale or foreign binary cannot run."""
    import shutil
    from miclip import _native
    for L in (_native.lib(), _native.lib_ab()):
        names = L.mi_build_sources().decode().split()
        assert "api.cpp" in names and "../../include/miclip.h" in names
        assert L.mi_build_id().decode() == _native.source_fingerprint(names)
    # a one-byte change in any source changes the fingerprint the loader compares
    names = _native.lib().mi_build_sources().decode().split()
    csrc = tmp_path / "pkg" / "csrc"   # (the header sits at ../../include/ from csrc/)
    csrc.mkdir(parents=True)
    for n in names:
        dst = csrc / n
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copyfile(os.path.join(_native.CSRC_DIR, n), dst)
    assert _native.source_fingerprint(names, str(csrc)) == _native.lib().mi_build_id().decode()
    with open(csrc / "rank.hip", "ab") as f:
        f.write(b" ")
    assert _native.source_fingerprint(names, str(csrc)) != _native.lib().mi_build_id().decode()


def test_weights_numel_matches_packer():
    from miclip import _native, config
    for name in ("test-tiny", "test-small", "ViT-B/32"):
        cfg = config.get_config(name)
        n = _native.lib().mi_clip_weights_numel(ctypes.byref(_native.Arch.from_config(cfg)))
        if name == "ViT-B/32":
            assert n == 151277313  # openai ViT-B/32 parameter count
        assert n == sum(np.asarray(v).size for v in state_dict(name).values())


def test_argument_errors_without_gpu():
    from miclip import _native
    L = _native.lib()
    rc = L.mi_rank_topk(None, 10, 512, 0, None, 1, (1 << 24) + 1, 0, 0, 0, None, None, None, 0, None)
    assert rc == -3 and b"k must be" in L.mi_last_error()
    rc = L.mi_rank_topk(None, 10, 512, 0, None, 1, 0, 0, 0, 0, None, None, None, 0, None)
    assert rc == -3 and b"k must be" in L.mi_last_error()
    rc = L.mi_rank_topk(None, 10, 500, 0, None, 1, 10, 0, 0, 0, None, None, None, 0, None)
    assert rc == -3 and b"multiple of 32" in L.mi_last_error()
    # the query block is staged in LDS: D is capped where it still fits
    rc = L.mi_rank_topk(None, 10, 1056, 0, None, 1, 10, 0, 0, 0, None, None, None, 0, None)
    assert rc == -3 and b"1024" in L.mi_last_error()
    rc = L.mi_rank_topk(None, 10, 1024, 0, None, 1, 10, 0, 0, 0, None, None, None, 0, None)
    assert rc == -1                                              # D = 1024 accepted; fails on the null pointers
    # large k (select + sort path) needs the score matrix in the workspace
    assert L.mi_rank_workspace_bytes(3000, 2, 200) >= 2 * 3000 * 4 + 2 * 2 * 256 * 8
    rc = L.mi_rank_merge(None, None, 1, 4, 0, 0, None, None, None)
    assert rc == -3
    arch = _native.Arch(512, 224, 12, 768, 32, 77, 49408, 512, 8, 12)
    ctx = ctypes.c_void_p()
    blob = np.zeros(10, np.float32)
    rc = L.mi_clip_create(ctypes.byref(arch), blob.ctypes.data, 10, 0, 1, ctypes.byref(ctx))
    assert rc == -1 and b"expected" in L.mi_last_error()
    rc = L.mi_clip_create(ctypes.byref(arch), blob.ctypes.data, 10, 0, 0, ctypes.byref(ctx))    # MI_F32: accepted
    assert rc == -1 and b"expected" in L.mi_last_error()
    rc = L.mi_clip_create(ctypes.byref(arch), blob.ctypes.data, 10, 0, 2, ctypes.byref(ctx))    # MI_F16: no
    assert rc == -3
    assert L.mi_rank_workspace_bytes(1_000_000, 32, 10) > 0


def test_missing_library_fails_loudly(monkeypatch):
    from miclip import _native
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", "/nonexistent/libmiclip.so")
    with pytest.raises(_native.MiClipError):
        _native.lib()


def test_no_cpu_execution_path():
    from miclip import api, _native
    with pytest.raises(RuntimeError):
        api.load("test-tiny", device="cpu")
    import miclip.model as M
    from miclip import config
    with pytest.raises(_native.MiClipError):
        M.CLIP(config.get_config("test-tiny"), state_dict("test-tiny"), device="cpu")


def test_mirror_certificate_delta_covers_worst_case():
    """The mirror certificate's |s_mirror - s_exact| bound (rank_mirror.hip
    mirror_delta) against the analytic worst case per unit |q|: fp16 RNE of a
    unit row (unit roundoff 2^-11), the query split (2^-22 with the
    hi/lo split, 2^-11 hi only), f32 accumulation of both dot products
    (2 gamma_D, gamma_D = D u / (1 - D u), u = 2^-24) and the subnormal floor."""
    from miclip import _native
    L = _native.lib()
    fn = L.mi_debug_mirror_delta
    fn.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    u = 2.0 ** -24
    for D in (512, 768):
        for split in (1, 0):
            dr, da = ctypes.c_float(), ctypes.c_float()
            assert fn(D, split, ctypes.byref(dr), ctypes.byref(da)) == 0
            gamma = D * u / (1 - D * u)
            worst = 2.0 ** -11 + (2.0 ** -22 if split else 2.0 ** -11) + 2 * gamma + 2 * np.sqrt(D) * 2.0 ** -25
            assert dr.value >= worst, (D, split, dr.value, worst)
            assert da.value >= np.sqrt(D) * 2.0 ** -25


def test_cert_delta_covers_worst_case():
    """The certified rank pass's per-query bound (rank_cert.hip rank_cert_delta)
    against the analytic worst case per unit |q| at D = 512: the query split into
    bf16 q1 + q2 (residual 2^-18) and, f32 rows, the row split c_hi + c_lo plus
    the dropped c_lo q2 (2^-18 each); the bf16 MFMA path's f32 accumulation of
    P = 2 D / 3 D products (gamma_P, doubled for internal truncation) and the
    exact chain's gamma_D; the two sums of squares (gamma_D relatively, halved by
    the square root) with the sqrt / reciprocal roundings; the subnormal floor."""
    from miclip import _native
    L = _native.lib()
    fn = L.mi_debug_cert_delta
    fn.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    u, D = 2.0 ** -24, 512

    def gamma(n):
        return n * u / (1 - n * u)

    for dt, P, split in ((0, 3 * D, 3 * 2.0 ** -18), (1, 2 * D, 2.0 ** -18)):
        dr, da = ctypes.c_float(), ctypes.c_float()
        assert fn(dt, ctypes.byref(dr), ctypes.byref(da)) == 0
        worst = split + 2 * gamma(P) + gamma(D) + gamma(D) + 4 * u + 2 * np.sqrt(D) * 2.0 ** -25
        assert dr.value >= worst, (dt, dr.value, worst)
        assert da.value >= np.sqrt(D) * 2.0 ** -25
    assert fn(2, ctypes.byref(ctypes.c_float()), ctypes.byref(ctypes.c_float())) != 0


def test_host_gather_concatenates_pieces():
    """mi_host_gather (host only): pieces of bytes objects, at offsets, in order,
    on 1 and 16 threads, byte ranges split across threads."""
    import ctypes
    from miclip import _native
    L = _native.lib()
    rng = np.random.default_rng(0)
    pieces = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 300_000, 40)]
    skip = [int(x) for x in rng.integers(0, 100, 40)]
    want = b"".join(p[min(s, len(p)):] for p, s in zip(pieces, skip))
    ptrs = np.array([ctypes.cast(ctypes.c_char_p(p), ctypes.c_void_p).value + min(s, len(p)) for p, s in zip(pieces, skip)],
                    np.uint64)
    lens = np.array([len(p) - min(s, len(p)) for p, s in zip(pieces, skip)], np.int64)
    for threads in (1, 16):
        out = np.zeros(len(want), np.uint8)
        assert L.mi_host_gather(out.ctypes.data, ptrs.ctypes.data, lens.ctypes.data, len(pieces), threads) == 0
        assert out.tobytes() == want
    assert L.mi_host_gather(None, None, None, 1, 1) == -1
