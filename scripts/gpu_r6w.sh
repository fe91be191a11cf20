# r06 w: PMC of the MX-fp8 c_fc GEMM (configs[4] pass shape) -- persistent vs per-tile kernel: where
# the waves' cycles go (waits, issue stalls, scalar / branch / LDS instructions, MFMA busy)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6w; mkdir -p $D
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d $D/p1 -o p1 -- python3 scripts/mx_persist_micro.py 2 fc8 > $D/p1.log 2>&1 || { tail -5 $D/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
  --output-format csv -d $D/p2 -o p2 -- python3 scripts/mx_persist_micro.py 2 fc8 > $D/p2.log 2>&1 || { tail -5 $D/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SMEM SQ_IFETCH GRBM_GUI_ACTIVE \
  --output-format csv -d $D/p3 -o p3 -- python3 scripts/mx_persist_micro.py 2 fc8 > $D/p3.log 2>&1 || { tail -5 $D/p3.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/r6w/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm_mx" not in k: continue
        k = re.search(r"(gemm_mx\w*kernel<[^>]*>)", k).group(1)
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {sum(v)/len(v):16.5g}")
PY
echo done
