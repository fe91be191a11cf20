"""The fp32 tower's S <= 64 attention (mi_op_attention_f32) at the bench's pass (10k ViT-B/32
frames, S = 50, W = 768): the product kernel (split-f16 operands, round 6) against the exact-f32 forms:
batched loads (A/B MICLIP_ATTN_F32_V=4), the round-5 kernel (=2), the one-wave-per-SIMD prefetch kernel (=3), interleaved, HIP events, outputs compared.
usage: python scripts/attn_f32_micro.py [frames] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))

import torch  # noqa: E402

from miclip import _native as N  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    S, W = 50, 768
    dev = torch.device("cuda:0")
    sp = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(3)
    qkv = torch.randn(B * S, 3 * W, device=dev, generator=g) * 2
    outs = {k: torch.empty(B * S, W, device=dev) for k in ("split", "batched", "in_loop", "prefetch")}
    L = N.lib_ab()

    def run(k):
        os.environ["MICLIP_ATTN_F32_V"] = {"split": "0", "batched": "4", "in_loop": "2", "prefetch": "3"}[k]
        N.check(L.mi_op_attention_f32(qkv.data_ptr(), outs[k].data_ptr(), B, S, W, 0, sp), "attn f32")
    for k in outs:
        run(k)
    torch.cuda.synchronize()
    same = all(torch.equal(outs["batched"].view(torch.int32), outs[k].view(torch.int32)) for k in ("in_loop", "prefetch"))
    dev_max = ((outs["split"] - outs["batched"]).abs().max() / outs["batched"].abs().max()).item()
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
    nbytes = B * S * 4 * W * 4   # qkv read + att written, f32
    for k in outs:
        print(f"attention f32 {k:8s} B={B} S={S} W={W}: {best[k]:8.1f} us {nbytes / best[k] / 1e3:7.1f} GB/s", flush=True)
    print(f"exact-f32 forms bit-identical {same}; split-f16 vs exact max |diff| / max |out| {dev_max:.3e}", flush=True)


if __name__ == "__main__":
    main()
