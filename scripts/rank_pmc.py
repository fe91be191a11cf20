"""Short driver for PMC passes over the fused rank kernel: 1M x D f32 corpus,
Q = 32, k = 10, a few launches (run under rocprofv3 --pmc ...).

  python scripts/rank_pmc.py [D] [reps] [variant env, e.g. MICLIP_RANK_NW=8]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))

for a in sys.argv[3:]:
    k, v = a.split("=", 1)
    os.environ[k] = v

import torch  # noqa: E402
from miclip import retrieval  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(3)
corpus = torch.randn(1_000_000, D, device=dev, generator=g)
q = torch.nn.functional.normalize(torch.randn(32, D, device=dev, generator=g), dim=1)
for _ in range(reps):
    retrieval.rank_topk(corpus, q, 10)
torch.cuda.synchronize()
print("done", D, reps)
