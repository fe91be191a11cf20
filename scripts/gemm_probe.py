"""Where a persistent GEMM tile's time goes: runs the timing-probe variant (19,
gemm.hip gemm_ppp_kernel<EPI, true>) and reads each workgroup's s_memrealtime
stamps (100 MHz) of its third tile: main loop, epilogue (register work + store
issue), and the gap until the next tile's main loop starts (first-stage wait
and the group re-offset barriers).  usage: python scripts/gemm_probe.py [shapes,comma]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
os.environ.setdefault("MICLIP_LIB", "ab")   # A/B build: schedule variants, probes and MICLIP_* switches
sys.path.insert(0, os.path.join(os.path.dirname(ROOT), "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))

import torch  # noqa: E402

from gemm_micro import SHAPES  # noqa: E402
from miclip import _native as N  # noqa: E402


def main():
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else ["fc500", "qkv500"]
    L = N.lib()
    fn = L.mi_debug_gemm_probe
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    fn.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    sp = torch.cuda.current_stream().cuda_stream
    for name in only:
        M, Nn, K, epi = SHAPES[name]
        A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
        W = ((torch.rand(Nn, K, device=dev, generator=g) * 2 - 1) * K ** -0.5).bfloat16()
        bias = torch.rand(Nn, device=dev, generator=g)
        out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            N.check(L.mi_op_gemm(A.data_ptr(), W.data_ptr(), bias.data_ptr(), out.data_ptr(), M, Nn, K,
                                 epi | (19 << 8), sp), "gemm")
        torch.cuda.synchronize()
        buf = np.zeros(4096 * 4, np.uint64)
        N.check(fn(buf.ctypes.data, buf.size), "probe")
        t = buf.reshape(-1, 4).astype(np.int64)
        t = t[(t[:, 0] > 0) & (t[:, 3] > 0)]
        us = lambda x: x * 0.01  # noqa: E731
        main_ = us(t[:, 1] - t[:, 0]); epi_ = us(t[:, 2] - t[:, 1]); gap = us(t[:, 3] - t[:, 2])
        print(f"{name}: {len(t)} WGs  tile {us(t[:, 3] - t[:, 0]).mean():.2f} us = main {main_.mean():.2f} "
              f"(p10 {np.percentile(main_, 10):.2f} p90 {np.percentile(main_, 90):.2f}) + epilogue {epi_.mean():.2f} "
              f"+ next-tile start {gap.mean():.2f} (p90 {np.percentile(gap, 90):.2f})", flush=True)


if __name__ == "__main__":
    main()
