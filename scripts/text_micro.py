"""encode_text timing (32 queries, B/32 text tower; the bench's step) with the product library
against A/B variants of the small-M GEMM dispatch (MICLIP_SMALLM=t: 128 x 128 tiles below t
256-tiles; MICLIP_SMALL64=u: 64 x 64 tiles below u 128-tiles), interleaved in one process, HIP events.

  python scripts/text_micro.py [queries] [rounds]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_SYNTHETIC_WEIGHTS", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402
from miclip import _native, api, config, weights  # noqa: E402


def main():
    Q = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda:0")
    cfg = config.get_config("ViT-B/32")
    tk = torch.from_numpy(weights.synthetic_tokens(Q, cfg.context_length, cfg.vocab_size)).to(dev)
    table = {"prod": (_native.lib, None), "sm64": (_native.lib_ab, "64"), "t64_256": (_native.lib_ab, "64", "256"),
             "t64_1024": (_native.lib_ab, "64", "1024")}
    models = {}

    def use(k):
        _native.lib = table[k][0]
        os.environ.pop("MICLIP_SMALLM", None)
        os.environ.pop("MICLIP_SMALL64", None)
        if table[k][1]:
            os.environ["MICLIP_SMALLM"] = table[k][1]
        if len(table[k]) > 2:
            os.environ["MICLIP_SMALL64"] = table[k][2]   # 64 x 64 tiles below that many 128 x 128 tiles

    for k in table:
        use(k)
        models[k], _ = api.load("ViT-B/32", device=dev)
    outs = {}
    for k, m in models.items():
        use(k)
        outs[k] = m.encode_text(tk, out_dtype=torch.float32).cpu().numpy()
    for k, o in outs.items():
        print(k, "max |diff| vs prod", float(np.abs(o - outs["prod"]).max()), flush=True)
    times = {k: [] for k in models}
    stream = torch.cuda.current_stream(dev)
    for _ in range(rounds):
        for k, m in models.items():
            use(k)
            m.encode_text(tk)
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(10):
                m.encode_text(tk)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            times[k].append(e0.elapsed_time(e1) * 100)
    for k, t in times.items():
        print(f"{k}: encode_text {Q} queries {min(t):.1f} us", flush=True)


if __name__ == "__main__":
    main()
