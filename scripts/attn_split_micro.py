"""The fp32 tower's S <= 64 attention writing out_proj's split operand (mi_op_attention_f32_split,
role 2) at the bench's pass (10k ViT-B/32 frames): the product kernel against the A/B form with
the bound's row-max load reduced late (MICLIP_F32_ATTN_LATE=1), and the f32-output kernel for
reference; interleaved rounds, HIP events, split outputs compared byte for byte.
usage: python scripts/attn_split_micro.py [frames] [reps]"""
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
    rmax = qkv[:, 2 * W:].abs().amax(dim=1).contiguous()
    out = {k: torch.zeros(B * S, 2 * W, dtype=torch.int16, device=dev) for k in ("prod", "late")}
    sc = {k: torch.zeros(B * S, device=dev) for k in out}
    f32 = torch.empty(B * S, W, device=dev)
    P, A = N.lib(), N.lib_ab()

    def run(k):
        if k == "f32":
            N.check(P.mi_op_attention_f32(qkv.data_ptr(), f32.data_ptr(), B, S, W, 0, sp), "attn")
            return
        os.environ["MICLIP_F32_ATTN_LATE"] = "1" if k == "late" else "0"
        L = A if k == "late" else P
        N.check(L.mi_op_attention_f32_split(qkv.data_ptr(), rmax.data_ptr(), 1.0, 0.0, out[k].data_ptr(), 2,
                                           sc[k].data_ptr(), B, S, W, 0, sp), "attn split")
    ks = ("prod", "late", "f32")
    for k in ks:
        run(k)
    torch.cuda.synchronize()
    same = torch.equal(out["prod"], out["late"]) and torch.equal(sc["prod"], sc["late"])
    best = {k: 1e30 for k in ks}
    for _ in range(3):
        for k in ks:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run(k)
            e1.record()
            torch.cuda.synchronize()
            best[k] = min(best[k], e0.elapsed_time(e1) * 1e3 / reps)
    for k in ks:
        print(f"attention f32 ({k:4s}) B={B} S={S} W={W}: {best[k]:8.1f} us", flush=True)
    print(f"split outputs identical {same}", flush=True)


if __name__ == "__main__":
    main()
