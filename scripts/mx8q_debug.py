"""Debug: the 8-phase MX kernel vs the 16x16x128 kernel on crafted operands
(unit scales, then random scales); prints where outputs differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_LIB", "ab")   # A/B build: schedule variants, probes and MICLIP_* switches
import torch  # noqa: E402
from miclip import _native as N  # noqa: E402

L = N.lib()
dev = torch.device("cuda:0")
sp = torch.cuda.current_stream().cuda_stream
M, Nn, K = 512, 256, 512
g = torch.Generator(device="cpu").manual_seed(1)
codes = torch.tensor([0x38, 0xb8, 0x30, 0x40, 0x00, 0x3c], dtype=torch.uint8)   # +-1, 0.5, 2, 0, 1.5
for mode in ("unit", "random"):
    qa = codes[torch.randint(0, 6, (M, K), generator=g)].to(dev)
    qw = codes[torch.randint(0, 6, (Nn, K), generator=g)].to(dev)
    if mode == "unit":
        sa = torch.full(((K // 128) * M * 2,), 127, dtype=torch.uint8, device=dev)
        sw = torch.full(((K // 128) * Nn * 2,), 127, dtype=torch.uint8, device=dev)
    else:
        sa = torch.randint(124, 131, ((K // 128) * M * 2,), generator=g, dtype=torch.uint8).to(dev)
        sw = torch.randint(124, 131, ((K // 128) * Nn * 2,), generator=g, dtype=torch.uint8).to(dev)
    outs = []
    for v in (0, 1):
        o = torch.zeros(M, Nn, dtype=torch.float32 if False else torch.bfloat16, device=dev)
        N.check(L.mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), None, o.data_ptr(), M, Nn,
                                K, 0 | (v << 8), sp), "g")
        outs.append(o.float())
    torch.cuda.synchronize()
    d = (outs[0] != outs[1])
    print(mode, "differ:", int(d.sum()), "of", d.numel())
    if d.any():
        rows = d.any(1).nonzero().flatten()
        cols = d.any(0).nonzero().flatten()
        print(" rows", rows[:20].tolist(), "... n", rows.numel())
        print(" cols", cols[:40].tolist(), "... n", cols.numel())
        r, c = int(rows[0]), int(cols[0])
        print(" sample", outs[0][r, :8].tolist(), outs[1][r, :8].tolist())
        # ratio pattern
        ratio = (outs[0] / outs[1]).flatten()
        ok = torch.isfinite(ratio) & (outs[1].flatten() != 0)
        vals, cnt = torch.unique(ratio[ok].round(decimals=4), return_counts=True)
        top = cnt.argsort(descending=True)[:8]
        print(" ratios", [(float(vals[i]), int(cnt[i])) for i in top])
    ok = (outs[0] == outs[1]).float()
    blk = ok.reshape(M // 16, 16, Nn // 16, 16).mean(dim=(1, 3))   # [M/16, N/16]
    print(" correct fraction per 16x16 block (rows = 16-row blocks 0..31 of tile 0, cols = 16-col blocks):")
    for rb in range(min(32, M // 16)):
        print("  ", "".join("#" if x > 0.99 else ("." if x < 0.01 else "+") for x in blk[rb].tolist()))
    inner = ok.reshape(M // 16, 16, Nn // 16, 4, 4).mean(dim=(0, 2, 4))   # [row in block 16, col group 4]
    print(" within-block (row fr x col group g):", [[round(float(x), 2) for x in r] for r in inner])
    break
