"""Attention microbenchmark through mi_op_attention (random bf16 qkv, HIP events).
Shapes: the bench chunk of each tower.  Every S runs the flash kernel (K/V chunks in LDS) by default;
causal bit 8 selects the one-wave LDS-P kernel for S <= 96, bit 9 the chunk-streaming flash kernel for S > 64 (default there: K/V resident in LDS).  usage: python scripts/attn_micro.py [reps] [shape,shape...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_LIB", "ab")   # A/B build: schedule variants, probes and MICLIP_* switches

import torch  # noqa: E402

from miclip import _native as N  # noqa: E402

SHAPES = [("B/32", 2000, 50, 768, 0), ("B/32c", 10000, 50, 768, 0), ("text", 256, 77, 512, 1), ("L/14", 385, 257, 1024, 0),
          ("L/14@336", 173, 577, 1024, 0),
          # the bench chunks of configs[2] (L/14, 1667 frames) and configs[4] (L/14@336)
          ("L/14c", 1667, 257, 1024, 0), ("L/14@336c", 1000, 577, 1024, 0)]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    L = N.lib()
    dev = torch.device("cuda:0")
    sp = torch.cuda.current_stream().cuda_stream
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    for name, B, S, W, causal in SHAPES:
        if only and name not in only:
            continue
        qkv = (torch.randn(B * S, 3 * W, device=dev) * 1.5).bfloat16()
        outs = {}
        modes = ([0, "vb"] if S <= 64 and os.environ.get("ATTN_SHORT_MODES") == "vb" else
                 [0, 0x100, "short", "short2", "short3", "pipe4", "pipe8", "vb"] if S <= 64 else [0, 0x100] if S <= 96
                 else [0] + [f"v{i}" for i in os.environ.get("ATTN_VARS", "4,5,6,7,8,9,10").split(",")])
        # resident-K/V kernel variants (attention.hip): v1 8 waves one tile at a time, v2 8 waves
        # two tiles at a time, v3 16 waves one tile at a time.  Every mode is timed in 3
        # interleaved rounds and the best round is kept (the first kernel timed in a process
        # otherwise pays for the clock ramp: 755 vs 638 us for the same kernel, r04_ag / r04_ah).
        outs = {m: torch.empty(B * S, W, dtype=torch.bfloat16, device=dev) for m in modes}

        def run(mode):
            os.environ.pop("MICLIP_ATTN_SHORT", None)
            if mode in ("short", "short2", "short3", "pipe4", "pipe8", "vb"):
                os.environ["MICLIP_ATTN_SHORT"] = {"short": "1", "short2": "2", "short3": "3", "pipe4": "54", "pipe8": "58",
                                                   "vb": "6"}[mode]
                os.environ.pop("MICLIP_ATTN_VAR", None)
            elif isinstance(mode, str):
                os.environ["MICLIP_ATTN_VAR"] = mode[1:]
            else:
                os.environ.pop("MICLIP_ATTN_VAR", None)
            flag = 0 if isinstance(mode, str) else mode
            N.check(L.mi_op_attention(qkv.data_ptr(), outs[mode].data_ptr(), B, S, W, causal | flag, sp), "attn")
        times = {m: [] for m in modes}
        for m in modes:
            run(m)
        torch.cuda.synchronize()
        for _ in range(3):
            for m in modes:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    run(m)
                e1.record()
                torch.cuda.synchronize()
                times[m].append(e0.elapsed_time(e1) * 1e3 / reps)
        for mode in modes:
            us = min(times[mode])
            fl = 4.0 * B * S * S * W * (0.5 if causal else 1.0)
            by = B * S * 4 * W * 2
            d = (outs[mode].float() - outs[0].float()).abs().max().item()
            kind = {0: "default", "v1": "res 8w x1", "v11": "res 8w x1 unsplit", "v12": "res 8w x1 split", "v13": "res 8w split first", "v14": "res 8w Q ahead", "v2": "res 8w x2", "v3": "res 16w x1", "v4": "r32 8w x2", "v5": "r32 12w", "v6": "r32 12w stag1", "v7": "r32 12w stag2", "v8": "r32 12w noload", "v9": "r32 12w noexp", "v10": "r32 12w 2-phase", "short": "res 4w (S<=64)", "short2": "flash 2 heads/wg", "short3": "flash 1h occ-6", "pipe4": "pipe 4/CU", "pipe8": "pipe 8/CU", "vb": "flash V reads batched", 0x100: "one-wave", 0x200: "flash(chunked)"}[mode]
            print(f"{name:9s} {kind:16s} B={B} S={S} W={W}: {us:8.1f} us "
                  f"{fl / us / 1e6:6.1f} TFLOP/s {by / us / 1e3:7.1f} GB/s  maxdiff {d:.3g}", flush=True)

if __name__ == "__main__":
    main()
