"""MX-fp8 vs bf16 GEMM at the ViT-L/14@336px tower shapes (M ~ 100k token rows),
random operands, HIP events, interleaved in one process.
usage: python scripts/gemm_mx_micro.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_LIB", "ab")   # A/B build: schedule variants, probes and MICLIP_* switches

import torch  # noqa: E402

from miclip import _native as N  # noqa: E402

SHAPES = {"qkv": (99821, 3072, 1024, 0), "out": (99821, 1024, 1024, 0), "fc": (99821, 4096, 1024, 1),
          "fc8": (99821, 4096, 1024, 4),   # c_fc -> MX-fp8 (the tower's EPI_GELU_MX; bf16 leg: GELU bf16)
          "proj": (99821, 1024, 4096, 0), "long": (16384, 4096, 4096, 0)}
if os.environ.get("MX_MICRO_SHAPES"):
    SHAPES = {k: SHAPES[k] for k in os.environ["MX_MICRO_SHAPES"].split(",")}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    L = N.lib()
    dev = torch.device("cuda:0")
    sp = torch.cuda.current_stream().cuda_stream
    for name, (M, Nn, K, epi) in SHAPES.items():
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        W = ((torch.rand(Nn, K, device=dev) * 2 - 1) * K ** -0.5).bfloat16()
        bias = torch.rand(Nn, device=dev)
        qa = torch.empty(M, K, dtype=torch.uint8, device=dev)
        sa = torch.zeros((K // 128) * (M + 1) * 2, dtype=torch.uint8, device=dev)
        qw = torch.empty(Nn, K, dtype=torch.uint8, device=dev)
        sw = torch.zeros((K // 128) * Nn * 2, dtype=torch.uint8, device=dev)
        N.check(L.mi_op_quantize_mx(A.data_ptr(), qa.data_ptr(), sa.data_ptr(), M, K, sp), "q")
        N.check(L.mi_op_quantize_mx(W.data_ptr(), qw.data_ptr(), sw.data_ptr(), Nn, K, sp), "q")
        o1 = torch.empty(M, Nn, dtype=torch.bfloat16, device=dev)
        o2 = torch.empty(M, Nn, dtype=torch.bfloat16, device=dev)
        if epi == 4:   # e4m3 [M, N] then the output's scales
            o2 = torch.zeros((M * Nn + 255) // 256 * 256 + (Nn // 128) * (M + (M & 1)) * 2, dtype=torch.uint8, device=dev)
        runs = {
            "bf16": lambda: N.check(L.mi_op_gemm(A.data_ptr(), W.data_ptr(), bias.data_ptr(), o1.data_ptr(), M, Nn, K,
                                                 1 if epi == 4 else epi, sp), "g"),
            "mxfp8": lambda: N.check(L.mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(),
                                                     bias.data_ptr(), o2.data_ptr(), M, Nn, K, epi, sp), "g"),
            "mx_pp": lambda: N.check(L.mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(),
                                                     bias.data_ptr(), o2.data_ptr(), M, Nn, K, epi | (8 << 8), sp), "g"),
            "mx_v1": lambda: N.check(L.mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(),
                                                     bias.data_ptr(), o2.data_ptr(), M, Nn, K, epi | (1 << 8), sp), "g"),
            "quant_A": lambda: N.check(L.mi_op_quantize_mx(A.data_ptr(), qa.data_ptr(), sa.data_ptr(), M, K, sp), "q"),
        }
        for f in runs.values():
            f()
        torch.cuda.synchronize()
        best = {k: 1e30 for k in runs}
        for _ in range(3):
            for k, f in runs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    f()
                e1.record()
                torch.cuda.synchronize()
                best[k] = min(best[k], e0.elapsed_time(e1) * 1e3 / reps)
        fl = 2.0 * M * Nn * K
        rel = float("nan") if epi == 4 else ((o1.float() - o2.float()).norm() / o1.float().norm()).item()
        print(f"{name:5s} M={M} N={Nn} K={K}: bf16 {best['bf16']:8.1f} us {fl / best['bf16'] / 1e6:7.1f} TF | "
              f"mxfp8 {best['mxfp8']:8.1f} us {fl / best['mxfp8'] / 1e6:7.1f} TF | 8-phase {best['mx_pp']:8.1f} us "
              f"{fl / best['mx_pp'] / 1e6:7.1f} TF | 16x16x128 {best['mx_v1']:8.1f} us | quantize A {best['quant_A']:7.1f} us"
              f" | rel diff {rel:.3g}", flush=True)
        del A, W, qa, qw, o1, o2


if __name__ == "__main__":
    main()
