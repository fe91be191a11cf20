"""Kernel-level breakdown of one certified rank call (rocprofv3 --kernel-trace --stats):
1M x 512 f32 and bf16 rows, 32 queries, k = 10, 10 calls each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_LIB", "ab")

import torch  # noqa: E402
from miclip import retrieval  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    dts = {"f32": (torch.float32,), "bf16": (torch.bfloat16,)}.get(os.environ.get("RC_DT", ""),
                                                                   (torch.float32, torch.bfloat16))
    for dt in dts:
        corpus = torch.randn(int(os.environ.get("RC_N", 1_000_000)), 512, device=dev, generator=g).to(dt)
        q = torch.nn.functional.normalize(torch.randn(32, 512, device=dev, generator=g), dim=1)
        for _ in range(10):
            retrieval.rank_topk(corpus, q, 10)
        torch.cuda.synchronize()
        del corpus


if __name__ == "__main__":
    main()
