"""HBM traffic per GEMM launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes over `scripts/gemm_micro.py 1 <shapes>` (scripts/gpu_traffic.sh).

gemm_micro runs 4 dispatches per shape in the order given, so dispatch i of the
libmiclip kernels belongs to shapes[i // 4].  Units and gfx950 corrections
(MI355X_MICROARCH.md "HBM"): both counters are in KiB; FETCH_SIZE reports half
of the bytes of a 16-B/lane streaming read (the LDS-DMA operand loads are that
form), so it is doubled; WRITE_SIZE is exact for 16-B/lane streaming stores.

usage: python scripts/pmc_traffic.py <prof dir> <shapes,comma> <out.json>
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_micro import SHAPES  # noqa: E402


def per_dispatch(path):
    rows = {}
    for r in csv.DictReader(open(path)):
        if "miclip" not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        rows.setdefault(d, [r["Kernel_Name"].split("(")[0], 0.0])
        rows[d][1] += float(r["Counter_Value"])
    return [rows[d] for d in sorted(rows)]


def main():
    root, shapes, out = sys.argv[1], sys.argv[2].split(","), sys.argv[3]
    fetch = per_dispatch(os.path.join(root, "FETCH_SIZE", "run_counter_collection.csv"))
    write = per_dispatch(os.path.join(root, "WRITE_SIZE", "run_counter_collection.csv"))
    res = {}
    for i, name in enumerate(shapes):
        M, N, K, epi = SHAPES[name]
        f = [v for _, v in fetch[4 * i:4 * i + 4]]
        w = [v for _, v in write[4 * i:4 * i + 4]]
        fb = 2 * 1024 * sum(f) / len(f)
        wb = 1024 * sum(w) / len(w)
        alg = 2 * (M * K + N * K + M * N)
        res[name] = {"kernel": fetch[4 * i][0], "shape": [M, N, K], "epilogue": epi,
                     "fetch_bytes": round(fb), "write_bytes": round(wb), "traffic_bytes": round(fb + wb),
                     "algorithmic_bytes": alg, "traffic_over_algorithmic": round((fb + wb) / alg, 3),
                     "fetch_size_kib_raw": f, "write_size_kib_raw": w}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print(k, v["traffic_bytes"] / 1e6, "MB vs", v["algorithmic_bytes"] / 1e6, "MB alg",
              v["traffic_over_algorithmic"])


if __name__ == "__main__":
    main()
