"""Where a gemm_8q tile's time goes: runs the stamp probe (variant 119 =
gemm_8q_kernel<EPI, 9>) and reads, per workgroup and M-group, the s_memtime
stamps of its third tile: S0 tile start (first pair, phase 1), S1 after the
previous tile's epilogue was issued, S2 phase 1's MFMA section starts, S3 the
first pair's phase-4 wait passed, S4/S5 around the first pair's phase-8 wait
(the epilogue stores must have completed), S6 tile end; plus s_memrealtime at
S0 and S6 for the shader clock.  usage: python scripts/gemm_probe8q.py [shapes,comma]"""
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
    var = int(sys.argv[2]) if len(sys.argv) > 2 else 119   # 118: staggered start
    L = N.lib()
    fn = L.mi_debug_gemm8q_probe
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
        for _ in range(5):
            N.check(L.mi_op_gemm(A.data_ptr(), W.data_ptr(), bias.data_ptr(), out.data_ptr(), M, Nn, K,
                                 epi | (var << 8), sp), "gemm")
        torch.cuda.synchronize()
        buf = np.zeros(1024 * 2 * 9, np.uint64)
        N.check(fn(buf.ctypes.data, buf.size), "probe")
        t = buf.reshape(-1, 2, 9).astype(np.int64)
        t = t[(t[:, :, 0] > 0).all(1) & (t[:, :, 6] > 0).all(1)]
        clk = (t[:, 0, 6] - t[:, 0, 0]) / ((t[:, 0, 8] - t[:, 0, 7]) * 10.0)   # cycles per ns = GHz
        r0 = (t[:, 0, 7] - t[:, 0, 7].min()) * 0.01
        print(f"{name} v{var}: {len(t)} WGs, shader clock {np.median(clk):.3f} GHz (p10 {np.percentile(clk, 10):.3f}); "
              f"third-tile start spread over WGs (us): p10 {np.percentile(r0, 10):.2f} p50 {np.percentile(r0, 50):.2f} "
              f"p90 {np.percentile(r0, 90):.2f} max {r0.max():.2f}")
        for grp in (0, 1):
            s = t[:, grp, :]
            d = lambda i, j: np.median(s[:, j] - s[:, i])  # noqa: E731
            print(f"  group {grp}: tile {d(0, 6):.0f} cyc | epilogue issue S0-S1 {d(0, 1):.0f} | S1-S2 (P1 reads+barrier) "
                  f"{d(1, 2):.0f} | S2-S3 (P1..P4 wait) {d(2, 3):.0f} | S3-S4 {d(3, 4):.0f} | P8 wait S4-S5 {d(4, 5):.0f} "
                  f"| S5-S6 (rest of tile) {d(5, 6):.0f}", flush=True)


if __name__ == "__main__":
    main()
