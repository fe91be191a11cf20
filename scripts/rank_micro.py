"""A/B of the fused rank kernel variants in ONE process, interleaved rounds
(default: the certified pass + gated exact pass for >= 262144 rows at D = 512, else rank_reg
for D = 512 and rank_stream otherwise; MICLIP_RANK_CERT=0: the exact pass alone;
MICLIP_RANK_REG=0: rank_stream), HIP events on the launch stream.

  python scripts/rank_micro.py [rounds]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
os.environ.setdefault("MICLIP_LIB", "ab")   # A/B build: schedule variants, probes and MICLIP_* switches

import torch  # noqa: E402
from miclip import retrieval  # noqa: E402

# default: the certified pass (rank_cert.hip) where eligible (>= 262144 rows, D = 512, k <= 12);
# exact: MICLIP_RANK_CERT=0, the exact pass alone
VARIANTS = {"default": {}, "exact": {"MICLIP_RANK_CERT": "0"},
            "stream12": {"MICLIP_RANK_REG": "0", "MICLIP_RANK_NW": "12", "MICLIP_RANK_CERT": "0"},
            "nomfma": {"MICLIP_RANK_PROBE": "1", "MICLIP_RANK_CERT": "0"},
            # certified-pass timing probes (wrong results): no Gram MFMAs, no MFMAs, no list update
            "c_nogram": {"MICLIP_RANK_CERT_ABL": "1"}, "c_nomfma": {"MICLIP_RANK_CERT_ABL": "2"},
            "c_nolist": {"MICLIP_RANK_CERT_ABL": "3"}, "c_endput": {"MICLIP_RANK_CERT_ABL": "6"},
            "c_noput": {"MICLIP_RANK_CERT_ABL": "7"},
            # round-4 in-launch merge instead of the split merge (r05)
            "cert_any": {"MICLIP_RANK_CERT": "2"},   # the certified route at every size (default: >= 262144 rows)
            "inl": {"MICLIP_RANK_FOLD": "1"}, "exact_inl": {"MICLIP_RANK_CERT": "0", "MICLIP_RANK_FOLD": "1"}}
SHAPES = [(125_000, 512, 32, torch.float32), (250_000, 512, 32, torch.float32), (125_000, 512, 32, torch.bfloat16), (1_000_000, 512, 32, torch.float32),
          (1_000_000, 512, 32, torch.bfloat16), (1_000_000, 768, 32, torch.float32)]
if os.environ.get("RANK_MICRO_VARIANTS"):   # a comma list of the variants to time
    VARIANTS = {v: VARIANTS[v] for v in os.environ["RANK_MICRO_VARIANTS"].split(",")}
if os.environ.get("RANK_MICRO_SHAPES") == "cert":   # the certified pass's shapes only
    SHAPES = SHAPES[1:3]


def setenv(v):
    for k in ("MICLIP_RANK_STAGE1", "MICLIP_RANK_NW", "MICLIP_RANK_REG", "MICLIP_RANK_PROBE", "MICLIP_RANK_ILV",
              "MICLIP_RANK_PIPE", "MICLIP_RANK_SEED", "MICLIP_RANK_CERT", "MICLIP_RANK_CERT_ABL",
              "MICLIP_RANK_FOLD"):
        os.environ.pop(k, None)
    os.environ.update(VARIANTS[v])


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    res = {}
    for (N, D, Q, dt) in SHAPES:
        corpus = torch.randn(N, D, device=dev, generator=g).to(dt)
        q = torch.nn.functional.normalize(torch.randn(Q, D, device=dev, generator=g), dim=1)
        name = f"N{N // 1000}k_D{D}_{'f32' if dt == torch.float32 else 'bf16'}"
        ref = None
        for v in VARIANTS:           # parity across variants: identical indices and scores
            setenv(v)
            s, i = retrieval.rank_topk(corpus, q, 10)
            if ref is None:
                ref = (s.clone(), i.clone())
            elif "nomfma" not in v and not v.startswith("c_"):   # timing probes: no scores
                assert torch.equal(i, ref[1]) and torch.equal(s, ref[0]), (name, v)
        times = {v: [] for v in VARIANTS}
        stream = torch.cuda.current_stream(dev)
        for _ in range(rounds):
            for v in VARIANTS:
                setenv(v)
                retrieval.rank_topk(corpus, q, 10)
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(10):
                    retrieval.rank_topk(corpus, q, 10)
                e1.record(stream)
                torch.cuda.synchronize(dev)
                times[v].append(e0.elapsed_time(e1) * 100)
        nb = corpus.numel() * corpus.element_size()
        res[name] = {v: {"us": round(min(t), 1), "gbs": round(nb / min(t) / 1e3, 1)} for v, t in times.items()}
        print(name, json.dumps(res[name]), flush=True)
        del corpus
    print(json.dumps(res))


if __name__ == "__main__":
    main()
