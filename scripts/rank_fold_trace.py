"""Kernel-trace driver for the ranking pass (product library): rank_topk at the
rank_roofline shapes, 20 calls each, for `rocprofv3 --kernel-trace --stats`.
usage: python scripts/rank_fold_trace.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))

import torch  # noqa: E402
from miclip import retrieval  # noqa: E402

SHAPES = [(125_000, 512, 32, torch.float32), (1_000_000, 512, 32, torch.float32),
          (1_000_000, 512, 32, torch.bfloat16), (1_000_000, 768, 32, torch.float32)]


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    for (N, D, Q, dt) in SHAPES:
        corpus = torch.randn(N, D, device=dev, generator=g).to(dt)
        q = torch.nn.functional.normalize(torch.randn(Q, D, device=dev, generator=g), dim=1)
        for _ in range(20):
            retrieval.rank_topk(corpus, q, 10)
        torch.cuda.synchronize(dev)
        print(N, D, Q, dt, flush=True)
        del corpus


if __name__ == "__main__":
    main()
