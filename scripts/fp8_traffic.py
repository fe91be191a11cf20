"""MX-fp8 c_fc GEMM (configs[4]: ViT-L/14@336px, one 863-frame chunk = 497951 token
rows x 4096 x 1024, QuickGELU epilogue) launched 4 times after one warm-up, for
rocprofv3 --pmc passes (scripts/gpu_fp8_traffic.sh), and the summary of those passes.

  python scripts/fp8_traffic.py run                       # the workload
  python scripts/fp8_traffic.py summarize <prof dir> <out.json>

Traffic per launch = FETCH_SIZE x 2 + WRITE_SIZE (KiB counters; the guide's gfx950
correction for 16-B/lane streaming reads), algorithmic bytes = fp8 A + fp8 W + their
e8m0 scales + bf16 C; MFMA busy from the GRBM/SQ pass as scripts/pmc_traffic.py does."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M, N_, K = 497951, 4096, 1024


def run():
    sys.path.insert(0, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"))
    import torch
    from miclip import _native as N
    L = N.lib()
    dev = torch.device("cuda:0")
    sp = torch.cuda.current_stream().cuda_stream
    A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    W = ((torch.rand(N_, K, device=dev) * 2 - 1) * K ** -0.5).bfloat16()
    bias = torch.rand(N_, device=dev)
    qa = torch.empty(M, K, dtype=torch.uint8, device=dev)
    sa = torch.zeros((K // 128) * (M + 1) * 2, dtype=torch.uint8, device=dev)
    qw = torch.empty(N_, K, dtype=torch.uint8, device=dev)
    sw = torch.zeros((K // 128) * N_ * 2, dtype=torch.uint8, device=dev)
    N.check(L.mi_op_quantize_mx(A.data_ptr(), qa.data_ptr(), sa.data_ptr(), M, K, sp), "q")
    N.check(L.mi_op_quantize_mx(W.data_ptr(), qw.data_ptr(), sw.data_ptr(), N_, K, sp), "q")
    del A, W
    # the tower's c_fc epilogue: QuickGELU -> MX-fp8 codes + their scales (EPI_GELU_MX, round 6; round
    # 3-5 passes measured the bf16-output form, epilogue 1)
    epi = int(os.environ.get("FP8_TRAFFIC_EPI", "4"))
    if epi == 4:
        o = torch.empty((M * N_ + 255) // 256 * 256 + (N_ // 128) * ((M + 1) & ~1) * 2, dtype=torch.uint8, device=dev)
    else:
        o = torch.empty(M, N_, dtype=torch.bfloat16, device=dev)
    for _ in range(5):
        N.check(L.mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                o.data_ptr(), M, N_, K, epi, sp), "gemm_mx")
    torch.cuda.synchronize()


def _gemm_rows(path):
    rows = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "gemm" not in name or "miclip" not in name:
            continue
        d = int(r["Dispatch_Id"])
        rows.setdefault(d, {"name": name.split("(")[0]})
        rows[d][r["Counter_Name"]] = rows[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [rows[d] for d in sorted(rows)][1:]   # drop the warm-up launch


def summarize(prof, out):
    fetch = [r["FETCH_SIZE"] for r in _gemm_rows(os.path.join(prof, "FETCH_SIZE", "run_counter_collection.csv"))]
    write = [r["WRITE_SIZE"] for r in _gemm_rows(os.path.join(prof, "WRITE_SIZE", "run_counter_collection.csv"))]
    mf = _gemm_rows(os.path.join(prof, "MFMA", "run_counter_collection.csv"))
    kib = 1024.0
    traffic = sum(2 * f * kib + w * kib for f, w in zip(fetch, write)) / len(fetch)
    # one e8m0 scale per 64 k; the output: MX-fp8 codes + one scale per 64 columns (epilogue 4, the
    # tower's) or bf16 (epilogue 1)
    epi = int(os.environ.get("FP8_TRAFFIC_EPI", "4"))
    alg = M * K + N_ * K + (M + N_) * (K // 64) + (M * N_ + M * (N_ // 64) if epi == 4 else M * N_ * 2)
    busy = None
    if mf:
        g = sum(r.get("GRBM_GUI_ACTIVE", 0.0) for r in mf) / len(mf)
        b = sum(r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for r in mf) / len(mf)
        busy = b / ((g / 8.0) * 1024.0) if g else None
    res = {"shape": [M, N_, K], "kernel": "gemm_mx (MX-fp8 c_fc + QuickGELU, configs[4]; epilogue %d)" % epi, "epilogue": epi,
           "traffic_bytes": round(traffic), "algorithmic_bytes": alg, "traffic_over_alg": round(traffic / alg, 3),
           "fetch_bytes": round(sum(fetch) / len(fetch) * 2 * kib), "write_bytes": round(sum(write) / len(write) * kib),
           "mfma_busy": round(busy, 4) if busy is not None else None, "launches": len(fetch),
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / (GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES) "
                     "passes over scripts/fp8_traffic.py run"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2], sys.argv[3])
