"""GEMM microbenchmark through mi_op_gemm (random bf16 operands, HIP events).

usage: python scripts/gemm_micro.py [reps] [shapes,comma] [variants,comma]
Shapes: the four ViT-B/32 tower GEMMs at a 2000-frame chunk (M = 100000) and
a long-K case that isolates main-loop efficiency.  Variants are main-loop
schedules (gemm.hip; 0 = default); each variant's output is checked against
the first one and timed in interleaved rounds in ONE process (guide §5.4 rule 24).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_LIB", "ab")   # A/B build: schedule variants, probes and MICLIP_* switches

import torch  # noqa: E402

from miclip import _native as N  # noqa: E402

SHAPES = {
    "qkv": (100000, 2304, 768, 0),
    "out": (100000, 768, 768, 0),
    "fc": (100000, 3072, 768, 1),
    "proj": (100000, 768, 3072, 0),
    # the bench's default pass since round 1's chunk change: 5000 frames = 250k rows
    "qkv250": (250000, 2304, 768, 0),
    "out250": (250000, 768, 768, 0),
    "fc250": (250000, 3072, 768, 1),
    "proj250": (250000, 768, 3072, 0),
    # bench default since the single-pass change: 10000 frames = 500k rows
    "qkv500": (500000, 2304, 768, 0),
    "out500": (500000, 768, 768, 0),
    "fc500": (500000, 3072, 768, 1),
    "proj500": (500000, 768, 3072, 0),
    "long": (16384, 4096, 4096, 0),
    "qkv20k": (20000, 2304, 768, 0),
    "fc20k": (20000, 3072, 768, 1),
    # LayerNorm-folded product GEMMs of the bf16 vision tower (epi 6: in_proj after ln_1,
    # 7: c_fc + QuickGELU after ln_2): fp16 operands in the residual stream's half-slot
    # layout (lda = 2K), through mi_op_gemm_ln; variants do not apply
    "lnqkv500": (500000, 2304, 768, 6),
    "lnfc500": (500000, 3072, 768, 7),
    "lnfc1k": (1000, 3072, 768, 7), "lnfc40k": (40003, 3072, 768, 7),   # (few / odd tile counts per CU)
    "lnfcL": (428459, 4096, 1024, 7),   # ViT-L/14 c_fc (1667 frames x 257 tokens)
    "lnfcL2": (494468, 4096, 1024, 7),  # ViT-L/14 c_fc at configs[2]'s bench pass (1924 frames x 257)
    "lnfc481": (480800, 3072, 768, 7),  # ViT-B/32 c_fc at configs[3]'s bench pass (9616 frames x 50)
    "lnqkvL": (428459, 3072, 1024, 6),   # ViT-L/14 in_proj
    "lnqkv250": (250000, 2304, 768, 6),
    "lnqkv100": (100000, 2304, 768, 6), "lnfc100": (100000, 3072, 768, 7),
    "lnfc250": (250000, 3072, 768, 7),
    # residual add fused into out_proj / c_proj (epi 8, mi_op_gemm_residual: x16 half-slot stream
    # read + written in the epilogue, row partials, residual_finalize); variant 1 = the unfused
    # pair it replaces (mi_op_gemm bf16 out, then mi_op_residual_stats); v2 / v3 probes (no
    # statistics / no x16 loads; A/B build, MICLIP_RES_ABL)
    "resout500": (500000, 768, 768, 8),
    "resproj500": (500000, 768, 3072, 8),
    # K sweep at the fc shape (per-tile fixed cost = intercept)
    "fcK384": (100000, 3072, 384, 0),
    "fcK768": (100000, 3072, 768, 0),
    "fcK1536": (100000, 3072, 1536, 0),
    "fcK3072": (100000, 3072, 3072, 0),
}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else list(SHAPES)
    all_variants = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0]
    L = N.lib()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    sp = torch.cuda.current_stream().cuda_stream
    for name in only:
        # "<shape>_t": operands rounded to bf16's 8-bit significand (LN shapes: still fp16 values),
        # so the same kernel runs on fewer toggling mantissa bits (MFMA power / clock probe)
        trunc = name.endswith("_t")
        M, Nn, K, epi = SHAPES[name[:-2] if trunc else name]
        ln = epi in (6, 7)
        dt = torch.float16 if ln else torch.bfloat16
        # LN shapes: A is the fp16 half-slot stream [M, 2K] (row stride 2K, first half used)
        A = (torch.rand(M, 2 * K if ln else K, device=dev, generator=g) * 2 - 1)
        W = ((torch.rand(Nn, K, device=dev, generator=g) * 2 - 1) * K ** -0.5)
        if trunc:
            A, W = A.bfloat16().float(), W.bfloat16().float()
        A, W = A.to(dt), W.to(dt)
        bias = torch.rand(Nn, device=dev, generator=g)
        res = epi == 8
        variants = (all_variants if os.environ.get("LN_FLAGS") else [0]) if ln else (
            (all_variants if os.environ.get("RES_VARIANTS") else [0, 1, 2, 3, 5]) if res else all_variants)
        if os.environ.get("GEMM_MICRO_V0"):   # PMC passes (scripts/pmc_traffic.py): the product kernel only
            variants = [0]
        if res:
            x16 = (torch.rand(M, 2 * Nn, device=dev, generator=g) * 2 - 1).half()
            ps = torch.empty(M, Nn // 64, 2, device=dev)
            rs2 = torch.empty(M, 2, device=dev)
        if ln:
            colsum = W.float().sum(1)
            rs = torch.rand(M + 256, 2, device=dev, generator=g) + 0.5
        outs = {v: torch.zeros(M, Nn, device=dev, dtype=torch.bfloat16 if epi in (0, 1, 6, 7, 8) else torch.float32)
                for v in variants}

        def run(v):
            if res:   # (x16 grows by the GEMM output each call: timing only, outputs not compared)
                # v2 / v3: timing probes of the fused kernel without statistics / without x16 loads
                # v5: non-temporal x16 loads / stores; v9: the lagging group's epilogue early (F_BEARLY)
                os.environ["MICLIP_RES_ABL"] = {2: "11", 3: "12", 5: "13", 9: "14", 6: "15"}.get(v, "0")
                # v6-v8: start stagger of half / a quarter of the workgroups (phases:ticks at 100 MHz)
                os.environ["MICLIP_RES_STAGGER"] = {6: "2:1500", 7: "2:750", 8: "4:750"}.get(v, "")
                if v != 1:
                    N.check(L.mi_op_gemm_residual(x16.data_ptr(), 2 * Nn, A.data_ptr(), K, W.data_ptr(),
                                                  bias.data_ptr(), ps.data_ptr(), rs2.data_ptr(), M, Nn, K, sp),
                            "gemm_residual")
                else:
                    N.check(L.mi_op_gemm(A.data_ptr(), W.data_ptr(), bias.data_ptr(), outs[v].data_ptr(), M, Nn, K,
                                         0, sp), "gemm")
                    N.check(L.mi_op_residual_stats(x16.data_ptr(), outs[v].data_ptr(), rs2.data_ptr(), M, Nn, sp),
                            "residual_stats")
                return
            if ln:   # LN_FLAGS=1: variant v = gemm_8q epilogue flags (MICLIP_8Q_F, A/B build)
                # (+ 10000: the per-XCD claimed tile order, MICLIP_8Q_DYN=1; without LN_FLAGS the
                # process environment's MICLIP_8Q_DYN stands, for PMC passes)
                # (19999 / 200xx: the product kernel with tile-order group width -1 (m-major) / xx,
                # MICLIP_8Q_NG)
                if os.environ.get("LN_FLAGS"):
                    os.environ["MICLIP_8Q_DYN"] = "1" if 10000 <= v < 19999 else "0"
                    if v >= 19999:
                        os.environ["MICLIP_8Q_NG"] = str(v - 20000)
                    else:
                        os.environ.pop("MICLIP_8Q_NG", None)
                os.environ["MICLIP_8Q_F"] = str(v % 10000) if v < 19999 else "0"
                N.check(L.mi_op_gemm_ln(A.data_ptr(), 2 * K, rs.data_ptr(), W.data_ptr(), colsum.data_ptr(),
                                        bias.data_ptr(), outs[v].data_ptr(), M, Nn, K, epi - 6, sp), "gemm_ln")
                return
            sched = v
            if os.environ.get("LN_FLAGS"):   # variant v = gemm_8q epilogue flags (MICLIP_8Q_F)
                os.environ["MICLIP_8Q_F"] = str(v)
                sched = 0
            N.check(L.mi_op_gemm(A.data_ptr(), W.data_ptr(), bias.data_ptr(), outs[v].data_ptr(), M, Nn, K,
                                 epi | (sched << 8), sp), "gemm")
        for v in variants:
            run(v)
        torch.cuda.synchronize()
        ref = outs[variants[0]].float()
        times = {v: [] for v in variants}
        for _ in range(3):
            for v in variants:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    run(v)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) * 1e3 / reps)
        for v in variants:
            us = min(times[v])
            err = (outs[v].float() - ref).abs().max().item()
            print(f"{name:7s} v{v} M={M} N={Nn} K={K} epi={epi}: {us:9.1f} us {2.0 * M * Nn * K / us / 1e6:7.1f} "
                  f"TFLOP/s  maxdiff vs v{variants[0]} {err:.3g}", flush=True)
        del A, W, outs, ref
        if ln:
            del rs, colsum


if __name__ == "__main__":
    main()
