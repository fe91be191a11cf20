"""The persistent MX-fp8 ping-pong (gemm_mxppp_kernel, the default since round 6) against one
workgroup per tile (gemm_mxpp_kernel, MICLIP_MX_PERSIST=0 in the A/B build) at the configs[4]
pass shapes (ViT-L/14@336px, 863 frames x 577 tokens = 497951 rows): random operands, HIP events,
interleaved rounds in one process, outputs compared byte for byte.
usage: python scripts/mx_persist_micro.py [reps] [shapes,comma] [group widths,comma]
(group widths: the persistent kernel's tile order, MICLIP_MX_NG, -1 = m-major; each also compared;
 an entry "pP:G" runs MICLIP_MX_PERSIST=P with MICLIP_MX_NG=G -- P 2 = persistent whatever K)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))

import torch  # noqa: E402

from miclip import _native as N  # noqa: E402

M4 = 863 * 577
SHAPES = {"qkv": (M4, 3072, 1024, 0), "out": (M4, 1024, 1024, 0), "fc8": (M4, 4096, 1024, 4),
          "proj": (M4, 1024, 4096, 0), "fc8_100k": (99821, 4096, 1024, 4)}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else list(SHAPES)
    ngs = sys.argv[3].split(",") if len(sys.argv) > 3 else []
    L = N.lib_ab()
    dev = torch.device("cuda:0")
    sp = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(5)
    for name in only:
        M, Nn, K, epi = SHAPES[name]
        A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
        W = ((torch.rand(Nn, K, device=dev, generator=g) * 2 - 1) * K ** -0.5).bfloat16()
        bias = torch.rand(Nn, device=dev, generator=g)
        qa = torch.empty(M, K, dtype=torch.uint8, device=dev)
        sa = torch.zeros((K // 128) * (M + 1) * 2, dtype=torch.uint8, device=dev)
        qw = torch.empty(Nn, K, dtype=torch.uint8, device=dev)
        sw = torch.zeros((K // 128) * Nn * 2, dtype=torch.uint8, device=dev)
        N.check(L.mi_op_quantize_mx(A.data_ptr(), qa.data_ptr(), sa.data_ptr(), M, K, sp), "q")
        N.check(L.mi_op_quantize_mx(W.data_ptr(), qw.data_ptr(), sw.data_ptr(), Nn, K, sp), "q")
        del A, W
        if epi == 4:
            mk = lambda: torch.zeros((M * Nn + 255) // 256 * 256 + (Nn // 128) * (M + (M & 1)) * 2,  # noqa: E731
                                     dtype=torch.uint8, device=dev)
        else:
            mk = lambda: torch.zeros(M, Nn, dtype=torch.bfloat16, device=dev)  # noqa: E731
        outs = {"persistent": mk(), "per_tile": mk()}
        for ng in ngs:
            outs[f"ng{ng}"] = mk()

        def run(k):
            os.environ["MICLIP_MX_PERSIST"] = "0" if k == "per_tile" else "1"
            os.environ.pop("MICLIP_MX_NG", None)
            if k.startswith("ngp"):      # "ngpP:G"
                pp, gg = k[3:].split(":")
                os.environ["MICLIP_MX_PERSIST"] = pp
                os.environ["MICLIP_MX_NG"] = gg
            elif k.startswith("ng"):
                os.environ["MICLIP_MX_NG"] = k[2:]
            N.check(L.mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                    outs[k].data_ptr(), M, Nn, K, epi, sp), "gemm_mx")
        for k in outs:
            run(k)
        torch.cuda.synchronize()
        same = torch.equal(outs["persistent"].view(torch.uint8), outs["per_tile"].view(torch.uint8))
        best = {k: 1e30 for k in outs}
        for _ in range(3):
            for k in outs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    run(k)
                e1.record()
                torch.cuda.synchronize()
                best[k] = min(best[k], e0.elapsed_time(e1) * 1e3 / reps)
        fl = 2.0 * M * Nn * K
        print(f"{name:8s} M={M} N={Nn} K={K} epi={epi}: persistent {best['persistent']:8.1f} us "
              f"{fl / best['persistent'] / 1e6:7.1f} TF ({fl / best['persistent'] / 1e6 / 5000:.3f} of fp8 peak) | "
              f"per-tile {best['per_tile']:8.1f} us {fl / best['per_tile'] / 1e6:7.1f} TF | bit-identical {same}",
              flush=True)
        for ng in ngs:
            k = f"ng{ng}"
            eq = torch.equal(outs[k].view(torch.uint8), outs["per_tile"].view(torch.uint8))
            print(f"{name:8s}   group width {ng:>5s}: {best[k]:8.1f} us {fl / best[k] / 1e6:7.1f} TF "
                  f"({fl / best[k] / 1e6 / 5000:.3f} of fp8 peak) | bit-identical {eq}", flush=True)
        del qa, qw, outs


if __name__ == "__main__":
    main()
