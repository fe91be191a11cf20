"""The fp32 tower (the R@K parity mode, weights="fp32") on the split-f16 GEMMs: the product
library (the 8-phase kernel, gemm_8q.hip's SPL epilogues) against the A/B library with
MICLIP_F32_8Q=0 (the ping-pong kernel), interleaved rounds in ONE process, HIP events on the
launch stream; outputs compared bit for bit.

  python scripts/f32_micro.py [frames] [rounds]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_SYNTHETIC_WEIGHTS", "1")   # random-init weights of the architecture

import numpy as np  # noqa: E402
import torch  # noqa: E402
from miclip import _native, api, config, weights  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda:0")
    cfg = config.get_config("ViT-B/32")
    px = torch.from_numpy(weights.synthetic_pixels(n, cfg.image_resolution)).to(dev)
    # variants: library + A/B environment (F32_VARIANTS=comma list; the first is the reference for bit-identity)
    table = {"8q": (_native.lib, {}), "pp": (_native.lib_ab, {"MICLIP_F32_8Q": "0"}),
             "bearly": (_native.lib_ab, {"MICLIP_F32_8Q": "2"}),
             "ng1": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_8Q_NG": "1"}),
             "ng3": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_8Q_NG": "3"}),
             "ab8q": (_native.lib_ab, {"MICLIP_F32_8Q": "1"}),
             "attv1": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_ATTN_F32_V": "1"}),
             "nodup": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "0"}),
             "dup1": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "1"}),
             "dup2": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "2"}),
             "dup4": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "4"}),
             "dup8": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "8"}),
             "nocls": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_CLS_LAST": "0"}),
             "ppnocls": (_native.lib_ab, {"MICLIP_F32_8Q": "0", "MICLIP_CLS_LAST": "0"}),
             "A": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "0", "MICLIP_CLS_LAST": "0"}),
             "B": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "0", "MICLIP_CLS_LAST": "1"}),
             "C": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "15", "MICLIP_CLS_LAST": "0"}),
             "A2": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "0", "MICLIP_CLS_LAST": "0"}),
             "m1": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "0", "MICLIP_CLS_LAST": "0", "MICLIP_F32_8Q_MASK": "1"}),
             "m2": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "0", "MICLIP_CLS_LAST": "0", "MICLIP_F32_8Q_MASK": "2"}),
             "m4": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "0", "MICLIP_CLS_LAST": "0", "MICLIP_F32_8Q_MASK": "4"}),
             "d8": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_F32_DUP": "8", "MICLIP_CLS_LAST": "0"}),
             "noim2s": (_native.lib_ab, {"MICLIP_F32_8Q": "1", "MICLIP_IM2COL_SPLIT": "0"})}
    names = os.environ.get("F32_VARIANTS", "8q,pp").split(",")
    libs = {k: table[k][0] for k in names}

    def use(k):   # (a model's calls go to whichever library _native.lib names)
        _native.lib = table[k][0]
        for e in ("MICLIP_F32_8Q", "MICLIP_8Q_NG", "MICLIP_ATTN_F32_V", "MICLIP_F32_DUP", "MICLIP_CLS_LAST",
                  "MICLIP_F32_8Q_MASK", "MICLIP_IM2COL_SPLIT"):
            os.environ.pop(e, None)
        os.environ.update(table[k][1])

    models = {}
    for name in names:
        use(name)
        models[name], _ = api.load("ViT-B/32", device=dev, image_chunk=n, weights="fp32")
    outs = {}
    for k, m in models.items():
        use(k)
        outs[k] = m.encode_image(px).cpu().numpy()
    same = all(np.array_equal(outs[names[0]].view(np.int32), o.view(np.int32)) for o in outs.values())
    print("bit-identical:", same, {k: bool(np.array_equal(outs[names[0]].view(np.int32), o.view(np.int32)))
                                   for k, o in outs.items()}, flush=True)
    for k, o in outs.items():
        bad = np.where(~np.isfinite(o).all(axis=1))[0]
        if len(bad):
            print(k, "non-finite rows:", len(bad), bad[:10].tolist(), "...", bad[-5:].tolist(), flush=True)
    print("max |diff|:", {k: float(np.abs(o - outs[names[0]]).max()) for k, o in outs.items()},
          "rows differing:", {k: int((o != outs[names[0]]).any(axis=1).sum()) for k, o in outs.items()}, flush=True)
    times = {k: [] for k in models}
    stream = torch.cuda.current_stream(dev)
    for _ in range(rounds):
        for k, m in models.items():
            use(k)
            m.encode_image(px)
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(3):
                m.encode_image(px)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            times[k].append(e0.elapsed_time(e1) / 3)
    for k, t in times.items():
        ms = min(t)
        print(f"{k}: encode_image {n} frames {ms:.2f} ms = {n / ms * 1e3:.0f} frames/s  (rounds {[round(x, 2) for x in t]})",
              flush=True)
    if not same and not os.environ.get("F32_NO_EXIT"):
        sys.exit(1)


if __name__ == "__main__":
    main()
