"""Fused JPEG ingest (8192 reference frames, bench.jpeg_ingest_timing's GPU path) against the
first launch's size (miclip.jpeg.FIRST_SUB: the pipeline's unhidden head) and the launch size
(SUB_FRAMES), interleaved rounds in one process, best of 3.  usage: python scripts/jpeg_first_sub.py"""
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
import torch  # noqa: E402
from miclip import jpeg  # noqa: E402

dev = torch.device("cuda:0")
files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "ref_frames", "*.jpg")))
raw = [open(f, "rb").read() for f in files]
B = 8192
bufs = [raw[i % len(raw)] for i in range(B)]
VARIANTS = [(512, 2048), (256, 2048), (128, 2048), (256, 1024), (256, 4096)]
best = {v: 1e9 for v in VARIANTS}
for rnd in range(4):
    for fs, sf in VARIANTS:
        jpeg.FIRST_SUB, jpeg.SUB_FRAMES = fs, sf
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = [x for _, x in jpeg.decode_groups(bufs, dev, transform=(224, False, torch.bfloat16))]
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if rnd:
            best[(fs, sf)] = min(best[(fs, sf)], dt)
        del out
for (fs, sf), dt in best.items():
    print(f"FIRST_SUB {fs:4d} SUB_FRAMES {sf:4d}: {B / dt:9.1f} frames/s ({dt * 1e3:.1f} ms)", flush=True)
