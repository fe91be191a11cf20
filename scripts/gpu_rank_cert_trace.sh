cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/rc -o rc -- python3 scripts/rank_cert_trace.py > gpurun_out/prof/rc.log 2>&1 || exit $?
python3 - <<'PY'
import csv
r = list(csv.DictReader(open("gpurun_out/prof/rc/rc_kernel_stats.csv")))
for x in r:
    print(x["Name"][:90], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), "us")
PY
