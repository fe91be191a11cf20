"""HBM traffic per GEMM launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes over `scripts/gemm_micro.py 1 <shapes>` (scripts/gpu_traffic.sh).

gemm_micro runs 4 dispatches per shape in the order given, so dispatch i of the
libmiclip kernels belongs to shapes[i // 4].  Units and gfx950 corrections
(MI355X_MICROARCH.md "HBM"): both counters are in KiB; FETCH_SIZE reports half
of the bytes of a 16-B/lane streaming read (the LDS-DMA operand loads are that
form), so it is doubled; WRITE_SIZE is exact for 16-B/lane streaming stores.

With a third pass in <prof dir>/MFMA (`--kernel-trace --pmc GRBM_GUI_ACTIVE
SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES`), each shape also gets its MFMA
utilisation: SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over all SIMDs) over
(GRBM_GUI_ACTIVE / 8 XCDs) x 1024 SIMDs, and the shader clock that pass ran at
(GRBM_GUI_ACTIVE / 8 over the dispatch's duration in the kernel trace).

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
        # the GEMMs only: mi_op_gemm_residual's residual_finalize pass (M x W / 8 bytes read,
        # M x 8 written) is not part of the GEMM launch counted here
        if "miclip" not in r["Kernel_Name"] or "gemm" not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        rows.setdefault(d, [r["Kernel_Name"].split("(")[0], 0.0])
        rows[d][1] += float(r["Counter_Value"])
    return [rows[d] for d in sorted(rows)]


def mfma_pass(root):
    d = os.path.join(root, "MFMA")
    cnt = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(cnt):
        return None
    per = {}
    for r in csv.DictReader(open(cnt)):
        if "miclip" not in r["Kernel_Name"] or "gemm" not in r["Kernel_Name"]:
            continue
        c = per.setdefault(int(r["Dispatch_Id"]), {})
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    dur = {}
    kt = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(kt):
        for r in csv.DictReader(open(kt)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = []
    for k in sorted(per):
        c = per[k]
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * 1024) if cyc else None
        hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        out.append({"mfma_busy": busy, "clock_ghz": cyc / dur[k] / 1e9 if k in dur and dur[k] > 0 else None,
                    "us": dur[k] * 1e6 if k in dur else None,
                    "l2_hit": hit / (hit + miss) if hit is not None and miss is not None and hit + miss > 0 else None})
    return out


def main():
    root, shapes, out = sys.argv[1], sys.argv[2].split(","), sys.argv[3]
    fetch = per_dispatch(os.path.join(root, "FETCH_SIZE", "run_counter_collection.csv"))
    write = per_dispatch(os.path.join(root, "WRITE_SIZE", "run_counter_collection.csv"))
    mf = mfma_pass(root)
    res = {}
    for i, name in enumerate(shapes):
        M, N, K, epi = SHAPES[name]
        f = [v for _, v in fetch[4 * i:4 * i + 4]]
        w = [v for _, v in write[4 * i:4 * i + 4]]
        fb = 2 * 1024 * sum(f) / len(f)
        wb = 1024 * sum(w) / len(w)
        alg = 2 * (M * K + N * K + M * N)
        if epi in (6, 7):                 # LayerNorm-folded: + rs (8 B per row) + colsum / colc (8 B per column)
            alg += 8 * M + 8 * N
        if epi == 8:                      # residual fused: + the x16 read (2 B) + row partials (8 B per 64 columns)
            alg += 2 * M * N + M * N // 8
        res[name] = {"kernel": fetch[4 * i][0], "shape": [M, N, K], "epilogue": epi,
                     "fetch_bytes": round(fb), "write_bytes": round(wb), "traffic_bytes": round(fb + wb),
                     "algorithmic_bytes": alg, "traffic_over_algorithmic": round((fb + wb) / alg, 3),
                     "fetch_size_kib_raw": f, "write_size_kib_raw": w}
        if mf and len(mf) >= 4 * i + 4:
            m = [x for x in mf[4 * i:4 * i + 4] if x["mfma_busy"] is not None]
            if m:
                res[name]["mfma_busy"] = round(sum(x["mfma_busy"] for x in m) / len(m), 4)
                ck = [x["clock_ghz"] for x in m if x["clock_ghz"]]
                res[name]["clock_ghz_mfma_pass"] = round(sum(ck) / len(ck), 3) if ck else None
                hr = [x["l2_hit"] for x in m if x.get("l2_hit") is not None]
                if hr:
                    res[name]["l2_hit_rate"] = round(sum(hr) / len(hr), 4)
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print(k, v["traffic_bytes"] / 1e6, "MB vs", v["algorithmic_bytes"] / 1e6, "MB alg",
              v["traffic_over_algorithmic"], "fetch/operands", round(v["fetch_bytes"] / (2 * (SHAPES[k][0] * SHAPES[k][2]
              + SHAPES[k][1] * SHAPES[k][2])), 2), "mfma busy", v.get("mfma_busy"), "L2 hit", v.get("l2_hit_rate"))


if __name__ == "__main__":
    main()
