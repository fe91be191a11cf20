"""Where the GPU JPEG ingest's wall time goes (8192 reference frames by
default): header parse, the pinned staging copy + upload (jpeg._upload), the
device decode (mi_jpeg_decode_transform, fused, the default; or mi_jpeg_decode +
the resample with argument 2 = "two"), each synchronised (so the stages do not
overlap here as they do in the pipeline), measured by wrapping the stages of
miclip.jpeg.decode_groups.  usage: python scripts/jpeg_breakdown.py [frames] [fused|two]"""
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
import torch  # noqa: E402
from miclip import _native as N, jpeg  # noqa: E402
from miclip.preprocess import preprocess_frames  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
FUSED = (sys.argv[2] if len(sys.argv) > 2 else "fused") == "fused"
files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "ref_frames", "*.jpg")))
raw = [open(f, "rb").read() for f in files]
bufs = [raw[i % len(raw)] for i in range(B)]
dev = torch.device("cuda:0")
T = {}


def timed(name, fn):
    def w(*a, **k):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize(dev)
        T[name] = T.get(name, 0.0) + time.perf_counter() - t0
        return r
    return w


jpeg._upload = timed("upload (pinned copy + H2D)", jpeg._upload)
L = N.lib()
orig_decode = L.mi_jpeg_decode
orig_xform = L.mi_jpeg_decode_transform


class _Wrap:
    def __getattr__(self, n):
        if n == "mi_jpeg_decode":
            return timed("mi_jpeg_decode (device)", orig_decode)
        if n == "mi_jpeg_decode_transform":
            return timed("mi_jpeg_decode_transform (device)", orig_xform)
        return getattr(L, n)


for rep in range(3):
    T.clear()
    N._lib = _Wrap()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    heads = [jpeg.parse(b) for b in bufs]
    T["parse"] = time.perf_counter() - t0
    outs = []
    tf = (224, False, torch.bfloat16) if FUSED else None
    for idx, rgb in jpeg.decode_groups(bufs, dev, heads=heads, transform=tf):
        if FUSED:
            outs.append(rgb)
            continue
        t1 = time.perf_counter()
        outs.append(preprocess_frames(rgb, 224, out_dtype=torch.bfloat16))
        torch.cuda.synchronize(dev)
        T["resample"] = T.get("resample", 0.0) + time.perf_counter() - t1
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    N._lib = L
    del outs
    T = {k: round(v * 1e3, 1) for k, v in T.items()}
    T["other host"] = round(wall * 1e3 - sum(T.values()), 1)
    print(json.dumps({"frames": B, "path": "fused" if FUSED else "two-step", "wall_ms": round(wall * 1e3, 1),
                      "frames_per_s": round(B / wall, 1), "ms": T}))
