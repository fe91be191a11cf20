# r04 o: SQ counters of the fused JPEG ingest kernels (transform: LDS- or issue-bound?)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4o
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/prof4o/p1 -o run -- \
  python3 scripts/jpeg_breakdown.py 2048 fused > gpurun_out/prof4o/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof4o/p2 -o run -- \
  python3 scripts/jpeg_breakdown.py 2048 fused > gpurun_out/prof4o/p2.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections
for p in ("p1", "p2"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for r in csv.DictReader(open(f"gpurun_out/prof4o/{p}/run_counter_collection.csv")):
        n = r["Kernel_Name"].replace("void ", "").replace("miclip::(anonymous namespace)::", "").split("(")[0]
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
    for n, d in agg.items():
        if "transform" in n or "final" in n or "sync" in n or "idct" in n:
            print(p, n[:30], {k: f"{v:.3g}" for k, v in sorted(d.items())})
PY
