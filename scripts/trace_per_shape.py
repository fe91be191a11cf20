"""Per-(kernel, grid) durations from a rocprofv3 --kernel-trace CSV, so that a
kernel template launched at several shapes (tower GEMMs, text vs image) gets
one average per shape.  usage:
  python scripts/trace_per_shape.py <kernel_trace.csv> <out.json> [dominant-note]"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("miclip::(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*$", "", name)                      # drop the argument list
    return name.strip()


def main():
    src, dst = sys.argv[1], sys.argv[2]
    note = sys.argv[3] if len(sys.argv) > 3 else None
    agg = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(src)):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        k = f"{short(r['Kernel_Name'])} grid={grid}"
        agg[k][0] += 1
        agg[k][1] += dur
    out = {"source": f"rocprofv3 --kernel-trace ({src}); per (kernel, grid) durations"}
    if note:
        out["dominant"] = note
    for k, (n, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        if not k.startswith(("gemm", "attention", "residual", "ln_", "rank", "resample", "im2col", "vision",
                             "finalize", "eot", "text_embed", "quantize")):
            continue
        out[k] = {"calls": n, "avg_us": round(tot / n, 2), "total_us": round(tot, 1)}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main()
