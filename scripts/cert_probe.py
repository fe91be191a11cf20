"""Stamp probe of the certified rank pass's per-tile list update (A/B build,
MICLIP_RANK_CERT_ABL=5): per wave, cycles spent in the update block, tiles,
tiles with an update, sort-path updates, multi-candidate updates.  1M x 512,
32 queries, f32 and bf16 rows."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ["MICLIP_LIB"] = "ab"
os.environ["MICLIP_RANK_CERT_ABL"] = "5"

import numpy as np  # noqa: E402
import torch  # noqa: E402
from miclip import _native as N, retrieval  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    L = N.lib()
    fn = L.mi_debug_cert_probe
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for dt in (torch.float32, torch.bfloat16):
        corpus = torch.randn(1_000_000, 512, device=dev, generator=g).to(dt)
        q = torch.nn.functional.normalize(torch.randn(32, 512, device=dev, generator=g), dim=1)
        for _ in range(3):
            retrieval.rank_topk(corpus, q, 10)
        torch.cuda.synchronize()
        buf = np.zeros(256 * 4 * 5, np.uint64)
        assert fn(buf.ctypes.data, buf.size) == 0
        b = buf.reshape(256 * 4, 5).astype(np.float64)
        cyc, tiles, upd, srt, multi = (b[:, i] for i in range(5))
        print(f"{dt}: tiles/wave {tiles.mean():.1f}, update tiles {upd.mean():.1f}, sort-path {srt.mean():.2f}, "
              f"multi-insert {multi.mean():.2f}, cycles in update block/wave {cyc.mean():.0f} "
              f"({cyc.sum() / max(tiles.sum(), 1):.0f} per tile)", flush=True)
        del corpus


if __name__ == "__main__":
    main()
