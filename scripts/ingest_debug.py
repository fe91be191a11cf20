"""Debug: GPU JPEG decode of the reference frames at growing batch sizes (first wrong frame)."""
import glob, io, os, sys
sys.path.insert(0, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd")
import numpy as np, torch
from PIL import Image
from miclip import jpeg
files = sorted(glob.glob("tests/golden/ref_frames/*.jpg"))
raw = [open(f, "rb").read() for f in files]
refs = [torch.from_numpy(np.asarray(Image.open(io.BytesIO(b)).convert("RGB"))).cuda() for b in raw]
for B in (1024, 2048, 3072, 4096, 6144, 8192):
    out = jpeg.decode_batch([raw[i % 16] for i in range(B)], "cuda")
    bad = [i for i in range(B) if not torch.equal(out[i], refs[i % 16])]
    info = ""
    if bad:
        d = (out[bad[0]] != refs[bad[0] % 16]).any(-1)
        rows = d.any(1).nonzero().flatten()
        info = f"first bad {bad[0]} rows {rows[:3].tolist()}..{rows[-1:].tolist()} frac {d.float().mean().item():.3f}"
    print("decode", B, "bad", len(bad), info, flush=True)
    del out
    torch.cuda.empty_cache()
