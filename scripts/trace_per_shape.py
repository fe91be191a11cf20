"""Per-(kernel, grid) durations from a rocprofv3 --kernel-trace CSV, so that a
kernel template launched at several shapes (tower GEMMs, text vs image) gets
one average per shape.  The persistent GEMMs launch one workgroup per CU
whatever M, so one (kernel, grid) can hold two shapes -- the 500k-row tower
launch and the CLS-row last block's (M = frames) -- whose durations differ by
~40x: such groups are split at a tenth of their longest launch into
"[full]" and "[short]" entries (round 6: without the split the c_fc average
mixed 11 full launches per step with the 52-us CLS-row launch).  usage:
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
    durs = defaultdict(list)
    for r in csv.DictReader(open(src)):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        durs[f"{short(r['Kernel_Name'])} grid={grid}"].append(dur)
    agg = {}
    for k, d in durs.items():
        top = max(d)
        lo = [x for x in d if x < 0.1 * top]
        if lo and len(lo) < len(d):
            agg[k + " [full]"] = [x for x in d if x >= 0.1 * top]
            agg[k + " [short]"] = lo
        else:
            agg[k] = d
    out = {"source": f"rocprofv3 --kernel-trace ({src}); per (kernel, grid) durations, a group whose launches "
                     "differ by more than 10x split into [full] / [short]"}
    if note:
        out["dominant"] = note
    for k, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        if not k.startswith(("gemm", "attention", "attn", "residual", "ln_", "rank", "resample", "im2col", "vision",
                             "finalize", "eot", "text_embed", "quantize", "split", "layernorm")):
            continue
        out[k] = {"calls": len(d), "avg_us": round(sum(d) / len(d), 2), "min_us": round(min(d), 2),
                  "max_us": round(max(d), 2), "total_us": round(sum(d), 1)}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main()
