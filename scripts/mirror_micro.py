"""Mirrored-corpus ranking vs the exact f32 pass, one process, HIP events on the
launch stream (csrc/rank_mirror.hip).  Per shape: the mirror call alone
(mirror pass + merge + exact re-score of 16 candidates per query), the whole
MirroredCorpus.topk (certificate read back, exact pass for uncertified queries),
and rank_topk over the f32 master; results must be bit-identical.

  python scripts/mirror_micro.py [rounds]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_LIB", "ab")   # A/B build: schedule variants, probes and MICLIP_* switches

import torch  # noqa: E402
from miclip import _native as N, retrieval  # noqa: E402

SHAPES = [(125_000, 512, 32), (1_000_000, 512, 32), (1_000_000, 512, 1), (1_000_000, 768, 32),
          (1_000_000, 768, 1000)]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    stream = torch.cuda.current_stream(dev)
    res = {}
    for (n, d, nq) in SHAPES:
        corpus = torch.randn(n, d, device=dev, generator=g)
        q = torch.nn.functional.normalize(torch.randn(nq, d, device=dev, generator=g), dim=1)
        t0 = time.time()
        mc = retrieval.MirroredCorpus(corpus)
        torch.cuda.synchronize(dev)
        build_ms = (time.time() - t0) * 1e3
        s, i = mc.topk(q, 10)
        s0, i0 = retrieval.rank_topk(corpus, q, 10)
        assert torch.equal(i, i0) and torch.equal(s, s0), (n, d, nq)
        cert = mc.certified
        L = N.lib()
        out_s = torch.empty((nq, 10), dtype=torch.float32, device=dev)
        out_i = torch.empty((nq, 10), dtype=torch.int64, device=dev)
        cflag = torch.empty(nq, dtype=torch.int32, device=dev)
        ws = torch.empty(L.mi_rank_mirror_workspace_bytes(n, nq), dtype=torch.uint8, device=dev)

        def mirror_call():
            N.check(L.mi_rank_mirror(mc.mirror.data_ptr(), corpus.data_ptr(), n, d, 0, q.data_ptr(), nq, 10, 0,
                                     0, out_s.data_ptr(), out_i.data_ptr(), cflag.data_ptr(), ws.data_ptr(),
                                     ws.numel(), N.stream_ptr(dev)), "mi_rank_mirror")

        reps = 3 if nq >= 1000 else 10
        def variant(v, fn):
            def run():
                os.environ["MICLIP_MIRROR_VAR"] = v
                fn()
                os.environ.pop("MICLIP_MIRROR_VAR")
            return run

        fns = {"mirror_call": mirror_call, "mirror_topk": lambda: mc.topk(q, 10),
               "exact_f32": lambda: retrieval.rank_topk(corpus, q, 10),
               "mirror_v1_nopipe": variant("1", mirror_call), "mirror_v2_pf7": variant("2", mirror_call),
               "mirror_v3_ilv": variant("3", mirror_call)}
        times = {name: [] for name in fns}
        for _ in range(rounds):
            for name, fn in fns.items():
                fn()
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(reps):
                    fn()
                e1.record(stream)
                torch.cuda.synchronize(dev)
                times[name].append(e0.elapsed_time(e1) * 1e3 / reps)
        mbytes = n * d * 2
        name = f"N{n // 1000}k_D{d}_Q{nq}"
        r = {k: round(min(v), 1) for k, v in times.items()}
        r["mirror_gbs"] = round(mbytes / r["mirror_call"] / 1e3, 1)
        r["mirror_hbm_frac"] = round(mbytes / r["mirror_call"] / 1e6 / 8.0, 4)
        r["speedup_vs_exact"] = round(r["exact_f32"] / r["mirror_topk"], 2)
        r["certified"] = f"{cert}/{nq}"
        r["build_ms"] = round(build_ms, 1)
        res[name] = r
        print(name, json.dumps(r), flush=True)
        del corpus, mc
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
