"""Host image preprocessing: openai/CLIP ``_transform(n_px)`` and the
``compare_models.py`` variant.

  _transform: Resize(n_px, BICUBIC) on the short side -> CenterCrop(n_px) ->
              RGB -> ToTensor -> Normalize(CLIP mean/std)
              (used at Backend/embedding.py:46, embedding_service.py:406,475)
  squash:     Resize((n_px, n_px)) -> ToTensor -> Normalize
              (compare_models.py:387-391; torchvision's default interpolation
              there is BILINEAR)

``Transform`` is the reference's host path, restated on PIL + numpy with
torchvision's size arithmetic (short side scaled, long side truncated; crop
offsets rounded half to even) since torchvision is not installed here.

``preprocess_frames`` is the same transform on the GPU for a batch of decoded
frames: ``mi_preprocess_frames`` resamples with
Pillow's exact integer algorithm, so its output equals ``Transform``'s bit for
bit (tests/test_preprocess.py).  JPEG decoding stays on the host (PIL; there
is no GPU JPEG decoder in this image).
"""
from __future__ import annotations

import os

import numpy as np

MEAN = np.array([0.48145466, 0.4578275, 0.40821073], dtype=np.float32)
STD = np.array([0.26862954, 0.26130258, 0.27577711], dtype=np.float32)


def _to_tensor(img):
    import torch
    a = np.asarray(img.convert("RGB"), dtype=np.float32) / 255.0
    a = (a - MEAN) / STD
    return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))


class Transform:
    def __init__(self, n_px: int, squash: bool = False):
        self.n_px = n_px
        self.squash = squash

    def __call__(self, img):
        from PIL import Image
        n = self.n_px
        if self.squash:
            img = img.resize((n, n), Image.BILINEAR)
            return _to_tensor(img)
        w, h = img.size
        if w <= h:
            nw, nh = n, int(n * h / w)
        else:
            nw, nh = int(n * w / h), n
        if (nw, nh) != (w, h):
            img = img.resize((nw, nh), Image.BICUBIC)
        left = int(round((nw - n) / 2.0))
        top = int(round((nh - n) / 2.0))
        img = img.crop((left, top, left + n, top + n))
        return _to_tensor(img)

    def batch(self, images, device="cuda", out_dtype=None):
        """GPU path for a list of PIL images of ONE size: host decode/convert,
        one upload of the uint8 frames, ``preprocess_frames`` on the device."""
        import torch
        frames = np.stack([np.asarray(im.convert("RGB"), dtype=np.uint8) for im in images])
        t = torch.from_numpy(frames).to(device)
        return preprocess_frames(t, self.n_px, squash=self.squash, out_dtype=out_dtype or torch.float32)

    def __repr__(self):
        return f"Transform(n_px={self.n_px}, squash={self.squash})"


def preprocess_frames(frames, n_px: int = 224, squash: bool = False, out_dtype=None):
    """frames: uint8 CUDA tensor [B, H, W, 3] (RGB) -> [B, 3, n_px, n_px]
    (float32 or bfloat16) through ``mi_preprocess_frames``; no CPU fallback."""
    import torch
    from . import _native as N
    if out_dtype is None:
        out_dtype = torch.float32
    if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3:
        raise N.MiClipError("preprocess_frames expects a uint8 tensor [B, H, W, 3]")
    if frames.device.type != "cuda":
        raise N.MiClipError("preprocess_frames runs on the GPU; host preprocessing is Transform")
    frames = frames.contiguous()
    B, H, W, _ = frames.shape
    mode = N.MI_PREP_SQUASH if squash else N.MI_PREP_CLIP
    L = N.lib()
    out = torch.empty(B, 3, n_px, n_px, dtype=out_dtype, device=frames.device)
    nb = L.mi_preprocess_workspace_bytes(B, H, W, n_px, mode)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=frames.device)
    with torch.cuda.device(frames.device):
        N.check(L.mi_preprocess_frames(frames.data_ptr(), B, H, W, n_px, mode, out.data_ptr(),
                                       N.dtype_code(out_dtype), ws.data_ptr(), nb, N.stream_ptr(frames.device)),
                "mi_preprocess_frames")
    return out


DECODE_CHUNK = 8192
DECODE_BUDGET_GB = 32


def decode_chunk(batch_size: int) -> int:
    """Frames per load_frames call in the folder-ingest loops: the GPU JPEG
    decode runs one lane per frame, so its rate grows with the batch (2048
    frames ~5k frames/s, 8192 ~13k) while the encode keeps the
    caller's batch size; a multiple of it (``$MICLIP_DECODE_CHUNK`` overrides).
    What one decode launch holds on the device is bounded separately, by bytes
    (``decode_budget``), so large frames (1080p, 4K) decode in smaller launches."""
    n = int(os.environ.get("MICLIP_DECODE_CHUNK", DECODE_CHUNK))
    b = max(1, batch_size)
    return max(b, n // b * b)


def decode_budget() -> int:
    """Device bytes a GPU decode launch may hold (RGB output + coefficient
    workspace, ``jpeg.decoded_bytes``): ``$MICLIP_DECODE_BUDGET_GB``, default 32 GB
    (~4.6k 720p frames, ~500 4K frames per launch; HBM is 288 GB)."""
    return int(float(os.environ.get("MICLIP_DECODE_BUDGET_GB", DECODE_BUDGET_GB)) * (1 << 30))


def _budget_slices(sizes, budget):
    """Consecutive [a, b) ranges whose summed sizes stay within budget (at least one item each)."""
    a, n = 0, len(sizes)
    while a < n:
        b, used = a, 0
        while b < n and (b == a or used + sizes[b] <= budget):
            used += sizes[b]
            b += 1
        yield a, b
        a = b


def load_frames(paths, n_px: int = 224, device="cuda", squash: bool = False, out_dtype=None, threads: int = 8,
                strict: bool = False, gpu_decode=None):
    """Decode frame files and preprocess them on the GPU.  Returns
    ([len(paths), 3, n_px, n_px] tensor in path order, list of failed indices).

    Decode: baseline JPEGs on the GPU (``miclip.jpeg``, bit-identical to
    Pillow; the default, ``$MICLIP_JPEG_GPU=0`` or ``gpu_decode=False`` turns it
    off), everything else with Pillow on host threads (decoding releases the
    GIL).  Each same-size group of decoded uint8 frames is preprocessed in one
    launch.  A frame that cannot be read is left as zeros, as the reference's
    ingest does (Backend/services/embedding_service.py:476-480); with
    ``strict`` the decode error propagates instead (Backend/embedding.py:45 has
    no handler)."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from PIL import Image

    if gpu_decode is None:
        gpu_decode = os.environ.get("MICLIP_JPEG_GPU", "1") != "0"
    if gpu_decode and str(device).startswith("cuda"):
        from . import jpeg

        def read(p):
            try:
                with open(p, "rb") as f:
                    return f.read()
            except OSError as e:
                if strict:
                    raise
                print(f"Error preprocessing image {p}: {e}")
                return b""

        with ThreadPoolExecutor(max(1, threads)) as ex:
            bufs = list(ex.map(read, paths))
        heads = [jpeg.parse(b) for b in bufs]
        out = torch.zeros(len(paths), 3, n_px, n_px, dtype=out_dtype or torch.float32, device=device)
        failed = []
        # the fused decode + transform kernel (mi_jpeg_decode_transform: no RGB frames in HBM,
        # bit-identical to decode + preprocess_frames); $MICLIP_JPEG_FUSED=0 runs the two steps
        fused = os.environ.get("MICLIP_JPEG_FUSED", "1") != "0"
        tf = (n_px, squash, out.dtype) if fused else None
        for a, b in _budget_slices([jpeg.decoded_bytes(h) for h in heads], decode_budget()):
            # each geometry group's decoded frames go to the resampler as the decoder's own [B,H,W,3] buffer
            for idx, rgb in jpeg.decode_groups(bufs[a:b], device, heads=heads[a:b], transform=tf):
                idx = [a + i for i in idx]
                if rgb is None:
                    i = idx[0]
                    if strict:      # Pillow's own error
                        with Image.open(paths[i]) as im:
                            im.convert("RGB")
                    if bufs[i]:
                        print(f"Error preprocessing image {paths[i]}: cannot identify or decode image file")
                    failed.append(i)
                    continue
                res = rgb if fused else preprocess_frames(rgb, n_px, squash=squash, out_dtype=out.dtype)
                del rgb
                if idx == list(range(idx[0], idx[0] + len(idx))):
                    out[idx[0]:idx[0] + len(idx)] = res
                else:
                    out[torch.tensor(idx, device=out.device)] = res
        return out, sorted(failed)

    def load(p):
        try:
            with Image.open(p) as im:
                return np.asarray(im.convert("RGB"), dtype=np.uint8)
        except Exception as e:  # reference: print and substitute a zero frame
            if strict:
                raise
            print(f"Error preprocessing image {p}: {e}")
            return None

    with ThreadPoolExecutor(max(1, threads)) as ex:
        arrs = list(ex.map(load, paths))
    out = torch.zeros(len(paths), 3, n_px, n_px, dtype=out_dtype or torch.float32, device=device)
    groups = {}
    for i, a in enumerate(arrs):
        if a is not None:
            groups.setdefault(a.shape, []).append(i)
    for idx in groups.values():
        frames = torch.from_numpy(np.stack([arrs[i] for i in idx])).to(device)
        out[torch.tensor(idx, device=out.device)] = preprocess_frames(frames, n_px, squash=squash,
                                                                       out_dtype=out.dtype)
    return out, [i for i, a in enumerate(arrs) if a is None]
