"""Exact rank pass (rank_reg) time against corpus size: the fixed cost of one call.
   python scripts/rank_nscale.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_LIB", "ab")
os.environ.setdefault("MICLIP_RANK_CERT", "0")

import torch  # noqa: E402
from miclip import retrieval  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    q = torch.nn.functional.normalize(torch.randn(32, 512, device=dev, generator=g), dim=1)
    for N in (1000, 4000, 10000, 30000, 62500, 125000, 250000, 500000, 1000000):
        corpus = torch.randn(N, 512, device=dev, generator=g)
        retrieval.rank_topk(corpus, q, 10)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                retrieval.rank_topk(corpus, q, 10)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 100)
        print(f"N {N:8d}: {best:7.1f} us  {N * 2048 / best / 1e3:7.1f} GB/s", flush=True)
        del corpus


if __name__ == "__main__":
    main()
