"""Phase stamps of the exact rank pass (rank_reg, MICLIP_RANK_STAMP=1, A/B build): per workgroup
s_memrealtime (100 MHz) at entry, after the query load, after the stream, after fold_publish, at exit.
   python scripts/rank_stamp.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_LIB", "ab")
os.environ["MICLIP_RANK_CERT"] = "0"
os.environ["MICLIP_RANK_STAMP"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402
from miclip import _native as N_  # noqa: E402
from miclip import retrieval  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    q = torch.nn.functional.normalize(torch.randn(32, 512, device=dev, generator=g), dim=1)
    L = N_.lib_ab()
    L.mi_debug_rank_stamp.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for N in (10000, 125000, 1000000):
        corpus = torch.randn(N, 512, device=dev, generator=g)
        for _ in range(3):
            retrieval.rank_topk(corpus, q, 10)
        torch.cuda.synchronize()
        buf = np.zeros(256 * 10, dtype=np.uint64)
        assert L.mi_debug_rank_stamp(buf.ctypes.data, buf.size) == 0
        st = buf.reshape(256, 10).astype(np.int64)
        st = st[st[:, 0] > 0]
        t0 = st[:, 0].min()
        rel = (st - t0) / 100.0   # s_memtime ticks at 100 MHz -> us
        nwg = len(st)
        print(f"N {N}: {nwg} workgroups; us from the first entry (median / max over workgroups):")
        for i, name in enumerate(["entry", "queries loaded", "stream done", "published", "exit", "ticket"]):
            print(f"  {name:15s} {np.median(rel[:, i]):8.1f} {rel[:, i].max():8.1f}")
        last = st[st[:, 6] > st[:, 5]]   # this launch's reducer (older launches' stamps 6-9 linger)
        for row in last:
            r = (row - t0) / 100.0
            print(f"  group reducer: ticket {r[5]:.1f} slabs taken {r[9]:.1f} group merged {r[6]:.1f}"
                  + (f" final ticket {r[7]:.1f} final merged {r[8]:.1f}" if row[8] > row[6] else "") + f" exit {r[4]:.1f}")
        del corpus


if __name__ == "__main__":
    main()
