# certified rank pass: its GPU tests, the rank micro (exact vs certified), a kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests/test_gpu_rank.py -x -q --timeout 150 --timeout-method thread > gpurun_out/rank_cert_test.log 2>&1
rc=$?; tail -15 gpurun_out/rank_cert_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/rank_micro.py 3 > gpurun_out/rank_micro.log 2>&1 || exit $?
head -5 gpurun_out/rank_micro.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/rc -o rc -- python3 scripts/rank_cert_trace.py > gpurun_out/prof/rc.log 2>&1 || exit $?
python3 - <<'PY'
import csv
r = list(csv.DictReader(open("gpurun_out/prof/rc/rc_kernel_stats.csv")))
for x in r:
    if "miclip" in x["Name"] or "rocclr" in x["Name"]:
        print(x["Name"][:90], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), "us")
PY
