"""Folder ingest end to end (Backend/embedding.py flow, miclip.embedding):
JPEG files on disk -> GPU decode + resample -> encode_image (B/32 bf16,
synthetic weights) -> .npy, on the reference's 16 frames linked N times.
Compares decode chunks of 8192 (default) and 256 (one encode batch).

  python scripts/ingest_micro.py [N]
"""
import glob
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_SYNTHETIC_WEIGHTS", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402
from miclip import api, embedding  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "ref_frames", "*.jpg")))
    model, pre = api.load("ViT-B/32", device="cuda")
    res = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        src = os.path.join(d, "frames")
        os.makedirs(src)
        for i in range(n):
            os.symlink(files[i % len(files)], os.path.join(src, f"{i:06d}.jpg"))
        outs = {}
        for chunk in ("8192", "256", "8192"):
            os.environ["MICLIP_DECODE_CHUNK"] = chunk
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f = embedding.extract_and_save_embeddings_from_folder(src, "ViT-B/32", video_name=f"v{chunk}",
                                                                  output_dir=d, model=model, preprocess=pre)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            outs[chunk] = np.load(f)
            res[f"decode_chunk_{chunk}"] = {"frames": n, "seconds": round(dt, 3), "frames_per_s": round(n / dt, 1)}
            print(chunk, res[f"decode_chunk_{chunk}"], flush=True)
        res["identical_rows"] = bool(np.array_equal(outs["8192"], outs["256"]))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
