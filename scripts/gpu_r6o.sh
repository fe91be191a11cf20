# r06 o: PMC of the fp32 tower's S <= 64 attention (product in-loop kernel vs the A/B prefetch
# kernel) at 10k B/32 frames: where the waves' cycles go, and the bytes they fetch
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6o; mkdir -p $D
timeout -s KILL 60 rocprofv3 -L > $D/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d $D/p1 -o p1 -- python3 scripts/attn_f32_micro.py 10000 2 > $D/p1.log 2>&1 || { tail -5 $D/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
  --output-format csv -d $D/p2 -o p2 -- python3 scripts/attn_f32_micro.py 10000 2 > $D/p2.log 2>&1 || { tail -5 $D/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d $D/p3 -o p3 -- python3 scripts/attn_f32_micro.py 10000 2 > $D/p3.log 2>&1 || { tail -5 $D/p3.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/r6o/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "attn_f32" not in k: continue
        agg[k[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {sum(v)/len(v):16.4g}  (n={len(v)})")
PY
