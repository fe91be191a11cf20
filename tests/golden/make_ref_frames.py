"""Copy a real-frame fixture out of the reference (run in the build container,
which has ``/root/reference``; the GPU box only reads the copies).

  python tests/golden/make_ref_frames.py

The reference commits genuine openai/CLIP ViT-B/32 ``encode_image`` outputs
for its own frames: ``Backend/embedding/video_test_4_embeddings.npy`` ([387,512]
fp32, the CPU ``Backend/embedding.py`` path, UN-normalised) whose rows follow
the frames of ``Backend/static/processed_frames/video_test_4/`` in sorted
file-name order.  This script copies 16 of
those 1280x720 JPEG frames (every 24th in sorted order) unchanged, with their
rows, to ``tests/golden/ref_frames/`` — data only, so a GPU test can pin
``encode_image`` to the reference's real outputs when real weights are supplied
(``$CLIP_WEIGHTS``), and the GPU preprocessing to PIL on real JPEGs always.
"""
from __future__ import annotations

import os
import shutil

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC_FRAMES = "/root/reference/Backend/static/processed_frames/video_test_4"
SRC_ROWS = "/root/reference/Backend/embedding/video_test_4_embeddings.npy"
OUT = os.path.join(HERE, "ref_frames")
STEP, COUNT = 24, 16


def main():
    names = sorted(f for f in os.listdir(SRC_FRAMES) if f.lower().endswith((".jpg", ".jpeg", ".png")))
    rows = np.load(SRC_ROWS, allow_pickle=False)
    assert rows.shape[0] == len(names), (rows.shape, len(names))
    pick = list(range(0, STEP * COUNT, STEP))
    os.makedirs(OUT, exist_ok=True)
    for i in pick:
        shutil.copyfile(os.path.join(SRC_FRAMES, names[i]), os.path.join(OUT, names[i]))
    np.savez_compressed(os.path.join(OUT, "video_test_4_rows.npz"), names=np.array([names[i] for i in pick]),
                        positions=np.array(pick), rows=rows[pick].astype(np.float32))
    print(f"wrote {len(pick)} frames + rows to {OUT}")


if __name__ == "__main__":
    main()
