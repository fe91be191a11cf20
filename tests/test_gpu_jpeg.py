"""GPU JPEG decode (mi_jpeg_decode) against Pillow
itself — the reference's own decoder (Image.open(p).convert("RGB"),
Backend/services/embedding_service.py:472-480): every pixel of every frame must
be identical.  Cases: the 16 real frames of the reference's
Backend/static/processed_frames (1280x720 4:2:0, standard tables), Pillow-written
JPEGs at 4:4:4 / 4:2:2 / 4:2:0, qualities 10..100, odd sizes (partial MCUs,
1-pixel edges), restart markers, grayscale; files the device path hands back to
the host (progressive, PNG, truncated) decode as Pillow does (or fail as it does)."""
import glob
import io
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.abspath(__file__))


def _pil(buf):
    from PIL import Image
    with Image.open(io.BytesIO(buf)) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)


def _img(h, w, seed, mode="RGB"):
    from PIL import Image
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = 127 + 80 * np.sin(xx / 5.0 + seed) * np.cos(yy / 7.0) + rng.normal(0, 40, (h, w))
    arr = np.stack([base, np.roll(base, 3, 1) * 0.8, 255 - base], -1)
    arr = np.clip(arr, 0, 255).astype(np.uint8)
    im = Image.fromarray(arr)
    return im.convert("L") if mode == "L" else im


def _save(im, **kw):
    b = io.BytesIO()
    im.save(b, "JPEG", **kw)
    return b.getvalue()


def _check(bufs, expect_device=None, **kw):
    from miclip import jpeg
    got = jpeg.decode_batch(bufs, "cuda", **kw)
    for i, (b, g) in enumerate(zip(bufs, got)):
        ref = _pil(b)
        assert g is not None, i
        g = g.cpu().numpy()
        assert g.shape == ref.shape, (i, g.shape, ref.shape)
        bad = np.argwhere(g != ref)
        assert bad.size == 0, f"frame {i}: {len(bad)} bytes differ, first {bad[:3].tolist()}"
    if expect_device is not None:
        assert [jpeg.parse(b).supported for b in bufs] == expect_device


def test_reference_frames_bit_exact(gpu):
    files = sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg")))
    assert len(files) == 16
    _check([open(f, "rb").read() for f in files], expect_device=[True] * 16)


@pytest.mark.parametrize("subsampling", [0, 1, 2])
@pytest.mark.parametrize("quality", [10, 75, 100])
def test_synthetic_sampling_quality_bit_exact(gpu, subsampling, quality):
    bufs = [_save(_img(h, w, s), quality=quality, subsampling=subsampling)
            for s, (h, w) in enumerate([(37, 53), (64, 64), (17, 9), (1, 1), (241, 319), (16, 33)])]
    _check(bufs, expect_device=[True] * len(bufs))


@pytest.mark.parametrize("kw", [dict(restart_marker_blocks=1), dict(restart_marker_blocks=5),
                                dict(restart_marker_rows=1), dict(restart_marker_rows=3)])
def test_restart_markers_bit_exact(gpu, kw):
    bufs = [_save(_img(h, w, 7 + s), quality=85, **kw) for s, (h, w) in enumerate([(72, 100), (131, 47), (200, 256)])]
    for b in bufs:
        assert b.count(b"\xff\xdd") == 1
    _check(bufs, expect_device=[True] * len(bufs))


@pytest.mark.parametrize("n", [3, 7])
def test_per_image_huffman_tables(gpu, n):
    """optimize=True gives every image its own Huffman tables: 3 distinct sets
    are staged in LDS, 7 exceed the LDS budget (4) and are read from global
    memory through the per-frame set index."""
    from miclip import jpeg
    bufs = [_save(_img(96, 128, 20 + s), quality=50 + 7 * s, optimize=True) for s in range(n)]
    sets = {tuple(sorted((k, bytes(b), v) for k, (b, v) in jpeg.parse(x).huff.items())) for x in bufs}
    assert len(sets) == n
    _check(bufs, expect_device=[True] * n)


def test_per_frame_tables_without_index(gpu):
    """huff_idx = NULL (one table set per frame, global-memory tables) gives
    the same pixels as the deduplicated LDS path."""
    files = sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg")))[:3]
    bufs = [open(f, "rb").read() for f in files] + [_save(_img(720, 1280, 9), quality=80)]
    _check(bufs, dedupe=False)


def test_large_batch_beyond_32bit_dispatch(gpu):
    """4800 reference frames (4.4e9 output pixels): a single per-pixel dispatch
    would overflow the 32-bit work-item count (frames past ~4660 came out
    stale); the IDCT / colour launches are chunked.  Every frame must equal
    Pillow's decode."""
    import torch
    from miclip import jpeg
    files = sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg")))
    raw = [open(f, "rb").read() for f in files]
    refs = [torch.from_numpy(_pil(b)).cuda() for b in raw]
    B = 4800
    got = jpeg.decode_batch([raw[i % len(raw)] for i in range(B)], "cuda")
    bad = [i for i in range(B) if got[i] is None or not torch.equal(got[i], refs[i % len(raw)])]
    assert not bad, f"{len(bad)} frames differ, first {bad[:5]}"
    del got
    torch.cuda.empty_cache()


def test_grayscale_and_mixed_batch(gpu):
    bufs = [_save(_img(45, 61, 1, "L"), quality=90), _save(_img(45, 61, 2), quality=90),
            _save(_img(45, 61, 3, "L"), quality=40), _save(_img(30, 30, 4), quality=90, subsampling=1)]
    _check(bufs, expect_device=[True] * 4)


def test_host_fallbacks(gpu):
    from PIL import Image
    from miclip import jpeg
    prog = _save(_img(50, 70, 5), quality=80, progressive=True)
    png = io.BytesIO()
    _img(20, 30, 6).save(png, "PNG")
    good = _save(_img(50, 70, 8), quality=80)
    bufs = [prog, png.getvalue(), good]
    assert [jpeg.parse(b).supported for b in bufs] == [False, False, True]
    _check(bufs)
    trunc = good[:len(good) // 2]
    assert not jpeg.parse(trunc).supported
    got = jpeg.decode_batch([trunc, b"not an image"], "cuda")
    with pytest.raises(OSError):
        with Image.open(io.BytesIO(trunc)) as im:
            im.convert("RGB")
    assert got == [None, None]


def test_load_frames_gpu_decode_matches_host_path(gpu, tmp_path):
    """miclip.preprocess.load_frames: the GPU-decode route and the Pillow route
    give bit-identical preprocessed tensors (mixed JPEG / PNG / unreadable files,
    two frame sizes); the unreadable file is a zero frame in both."""
    import shutil
    import torch
    from miclip.preprocess import load_frames
    files = sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg")))[:5]
    paths = []
    for i, f in enumerate(files):
        paths.append(str(tmp_path / f"{i}.jpg"))
        shutil.copy(f, paths[-1])
    _img(90, 120, 3).save(tmp_path / "a.png")
    (tmp_path / "b.jpg").write_bytes(_save(_img(90, 120, 4), quality=70, subsampling=1))
    (tmp_path / "bad.jpg").write_bytes(b"\xff\xd8garbage")
    paths += [str(tmp_path / "a.png"), str(tmp_path / "b.jpg"), str(tmp_path / "bad.jpg")]
    for squash in (False, True):
        g, fg = load_frames(paths, 224, "cuda", squash=squash, gpu_decode=True)
        h, fh = load_frames(paths, 224, "cuda", squash=squash, gpu_decode=False)
        assert fg == fh == [len(paths) - 1]
        assert torch.equal(g, h)
        assert not g[-1].any()


def _serial_reference(bufs, monkeypatch):
    """The same batch through the A/B build's lane-per-frame entropy kernel
    (MICLIP_JPEG_SERIAL=1): the decode the chunked kernels must reproduce."""
    from miclip import _native, jpeg
    monkeypatch.setattr(_native, "lib", _native.lib_ab)
    monkeypatch.setenv("MICLIP_JPEG_SERIAL", "1")
    out = [None if g is None else g.cpu().numpy() for g in jpeg.decode_batch(bufs, "cuda")]
    monkeypatch.undo()
    return out


def _corrupt(buf, seed):
    """Flip bytes of the entropy-coded data (markers and stuffing included by
    chance), keeping the headers and the final EOI: still a device-path file."""
    from miclip import jpeg
    h = jpeg.parse(buf)
    b = bytearray(buf)
    rng = np.random.default_rng(seed)
    lo, hi = h.scan_start, len(b) - 2
    for i in rng.integers(lo, hi, size=1 + seed % 5):
        b[i] = int(rng.integers(0, 256))
    if seed % 3 == 0:                                 # a marker in the middle of the scan
        i = int(rng.integers(lo, hi - 2))
        b[i:i + 2] = b"\xff\xd3"
    return bytes(b)


def test_chunked_entropy_matches_serial_on_corrupt_and_truncated(gpu, monkeypatch):
    """The chunked (speculative, self-synchronising) entropy decode must give
    the serial decode's coefficients on ANY byte stream — corrupt codes, a
    marker mid-scan (zero feed from there), truncation — since its consistency
    rounds only accept exit states reached from the true entry state."""
    from miclip import jpeg
    base = [_save(_img(h, w, s), quality=q) for h, w, s, q in
            ((720, 1280, 1, 90), (480, 640, 2, 50), (1080, 1920, 3, 95), (64, 72, 4, 75), (8, 8, 5, 30))]
    ref_frames = sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg")))[:3]
    base += [open(f, "rb").read() for f in ref_frames]
    bufs = []
    for i, b in enumerate(base):
        bufs.append(_corrupt(b, i))
        h = jpeg.parse(b)
        cut = h.scan_start + (len(b) - h.scan_start) * (i + 1) // (len(base) + 2)
        bufs.append(b[:cut] + b"\xff\xd9")              # truncated mid-scan
    assert all(jpeg.parse(b).supported for b in bufs)
    ser = _serial_reference(bufs, monkeypatch)
    got = jpeg.decode_batch(bufs, "cuda")
    for i, (g, r) in enumerate(zip(got, ser)):
        assert g is not None and r is not None, i
        assert np.array_equal(g.cpu().numpy(), r), f"buffer {i}: chunked decode differs from the serial kernel"


@pytest.mark.parametrize("quality", [20, 75, 100])
def test_chunked_entropy_large_frames_bit_exact(gpu, quality):
    """1080p / 4K frames (hundreds of 1-KB chunks per frame, DC prediction
    carried across every chunk edge) against Pillow."""
    bufs = [_save(_img(1080, 1920, 7), quality=quality), _save(_img(2160, 3840, 8), quality=quality),
            _save(_img(1080, 1920, 9), quality=quality, subsampling=0)]
    _check(bufs, expect_device=[True, True, True])


def test_load_frames_decode_budget(gpu, monkeypatch):
    """Decode launches bounded by device bytes (MICLIP_DECODE_BUDGET_GB): a
    budget of ~2 frames splits 16 reference frames into 8 launches with the
    same output as one launch."""
    from miclip.preprocess import load_frames
    files = sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg")))
    one, bad1 = load_frames(files, 224)
    monkeypatch.setenv("MICLIP_DECODE_BUDGET_GB", str(2 * 7e6 / (1 << 30)))
    many, bad2 = load_frames(files, 224)
    assert bad1 == bad2 == [] and torch_equal(one, many)


def torch_equal(a, b):
    import torch
    return torch.equal(a, b)


def _decode_raw(bufs, order, off_fn):
    """mi_jpeg_decode through the C-ABI on the scans of ``bufs`` concatenated in
    order, with frame f reading the byte range off_fn(f, starts) -> (seg_off,
    seg_end) of that concatenation (``order`` maps frames to buffers)."""
    import torch
    from miclip import _native as N, jpeg
    heads = [jpeg.parse(b) for b in bufs]
    key = jpeg._geom_key(heads[0])
    segl = [((h.scan_start, len(b)),) for h, b in zip(heads, bufs)]
    geom, huff, hidx, qt, offs, ends, starts, nsets = jpeg.launch_args(bufs, heads, list(range(len(bufs))), segl, key)
    data = b"".join(b[h.scan_start:] for h, b in zip(heads, bufs))
    total = len(data)
    dev = torch.device("cuda")
    d_data = torch.frombuffer(bytearray(data + b"\xff\xd9" * 16), dtype=torch.uint8).to(dev)
    B = len(order)
    so = np.zeros(B, np.int64)
    se = np.zeros(B, np.int64)
    for f in range(B):
        so[f], se[f] = off_fn(f, order[f], starts)
    W, H = int(geom[0]), int(geom[1])
    rgb = torch.empty(B, H, W, 3, dtype=torch.uint8, device=dev)
    L = N.lib()
    nb = L.mi_jpeg_workspace_bytes(geom.ctypes.data, B, total)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    d_h = torch.from_numpy(huff.view(np.uint8).reshape(-1)).to(dev)
    d_i = torch.from_numpy(np.ascontiguousarray(hidx[list(order)])).to(dev)
    d_q = torch.from_numpy(np.ascontiguousarray(qt[list(order)])).to(dev)
    d_so, d_se = torch.from_numpy(so).to(dev), torch.from_numpy(se).to(dev)     # kept alive over the call
    N.check(L.mi_jpeg_decode(d_data.data_ptr(), total, d_so.data_ptr(), d_se.data_ptr(), d_h.data_ptr(), d_i.data_ptr(), nsets,
                             d_q.data_ptr(), geom.ctypes.data, B, rgb.data_ptr(), ws.data_ptr(), nb,
                             N.stream_ptr(dev)), "mi_jpeg_decode")
    torch.cuda.synchronize()
    return rgb.cpu().numpy()


def test_segments_outside_the_contract_stay_in_bounds(gpu):
    """mi_jpeg_decode's segments are meant to be disjoint, in frame order, inside
    [0, data_bytes).  Callers that break that must not make the
    chunked decode write past its workspace: the same scan referenced by two
    frames, frames out of order, and a segment end past data_bytes.  Those frames
    leave the chunk layout and are decoded by the serial kernel from the data
    (clipped to data_bytes), so every frame still equals Pillow."""
    files = sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg")))[:3]
    bufs = [open(f, "rb").read() for f in files]
    refs = [_pil(b) for b in bufs]
    rng = lambda i, st: (int(st[i]), int(st[i + 1]))
    # frame 1 repeats frame 0's bytes; frame 3 re-reads frame 1's (out of order); frame 4 runs past the end
    order = [0, 0, 1, 1, 2]
    specs = {0: lambda st: rng(0, st), 1: lambda st: rng(0, st), 2: lambda st: rng(1, st),
             3: lambda st: rng(1, st), 4: lambda st: (int(st[2]), int(st[3]) + 100_000)}
    got = _decode_raw(bufs, order, lambda f, b, st: specs[f](st))
    for f, b in enumerate(order):
        assert np.array_equal(got[f], refs[b]), f"frame {f}"
    # reversed order: every frame after the first starts before an earlier end
    got = _decode_raw(bufs, [2, 1, 0], lambda f, b, st: rng(b, st))
    for f, b in enumerate([2, 1, 0]):
        assert np.array_equal(got[f], refs[b]), f"reversed frame {f}"


@pytest.mark.parametrize("squash", [False, True])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_fused_decode_transform_bit_identical(gpu, squash, dtype):
    """mi_jpeg_decode_transform (colour conversion + both Pillow resample passes +
    crop + ToTensor/Normalize in one kernel over the component planes, no RGB
    frames in HBM) == mi_jpeg_decode + mi_preprocess_frames, bit for bit: the
    reference frames (1280x720 4:2:0), 4:4:4 / 4:2:2 / grayscale / restart
    markers / odd sizes, sources smaller than the output (upsampling), and 1080p /
    4K (narrower LDS bands), both transforms, f32 and bf16 outputs."""
    import torch
    from miclip import jpeg
    from miclip.preprocess import preprocess_frames
    files = sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg")))[:4]
    bufs = [open(f, "rb").read() for f in files]
    bufs += [_save(_img(h, w, s), quality=q, subsampling=sub) for h, w, s, q, sub in
             ((481, 641, 1, 90, 0), (333, 500, 2, 75, 1), (720, 1280, 3, 85, 2), (100, 60, 4, 80, 2),
              (1080, 1920, 5, 90, 2), (2160, 3840, 6, 70, 2))]
    bufs += [_save(_img(300, 400, 7, "L"), quality=80), _save(_img(256, 320, 8), quality=90, restart_marker_rows=1)]
    odt = torch.float32 if dtype == "f32" else torch.bfloat16
    for n in (224, 336):
        got = {}
        for idx, x in jpeg.decode_groups(bufs, "cuda", transform=(n, squash, odt)):
            for r, i in enumerate(idx):
                got[i] = x[r]
        for idx, rgb in jpeg.decode_groups(bufs, "cuda"):
            ref = preprocess_frames(rgb, n, squash=squash, out_dtype=odt)
            for r, i in enumerate(idx):
                a, b = got[i], ref[r]
                assert a.shape == b.shape == (3, n, n)
                assert torch.equal(a.view(torch.int16) if dtype == "bf16" else a.view(torch.int32),
                                   b.view(torch.int16) if dtype == "bf16" else b.view(torch.int32)), (n, i)


def test_load_frames_fused_matches_two_step(gpu, tmp_path, monkeypatch):
    """preprocess.load_frames through the fused kernel == the two-step path
    ($MICLIP_JPEG_FUSED=0), including a PNG and an unreadable file (zero frame)."""
    import torch
    from miclip import preprocess
    paths = []
    for i, f in enumerate(sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg")))[:5]):
        paths.append(f)
    png = tmp_path / "x.png"
    _img(90, 160, 3).save(png)
    paths.append(str(png))
    bad = tmp_path / "bad.jpg"
    bad.write_bytes(b"not a jpeg")
    paths.append(str(bad))
    a, fa = preprocess.load_frames(paths, 224, device="cuda", out_dtype=torch.bfloat16)
    monkeypatch.setenv("MICLIP_JPEG_FUSED", "0")
    b, fb = preprocess.load_frames(paths, 224, device="cuda", out_dtype=torch.bfloat16)
    assert fa == fb == [len(paths) - 1]
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
