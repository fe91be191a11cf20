# r04 q: one fill per certified rank call (unsafe flag in the fold counters' memset; the re-score
# clears the gated exact pass's counters): rank tests, the call's kernel timeline, rank_micro
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4q
timeout -k 10 900 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_rank_scale.py tests/test_gpu_distributed.py tests/test_gpu_service.py tests/test_gpu_flows.py -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/r4q_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4q_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof4q/rc -o rc -- python3 scripts/rank_cert_trace.py > gpurun_out/prof4q/rc.log 2>&1 || exit $?
python3 - <<'PY'
import csv
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("void ", "").replace("miclip::(anonymous namespace)::", "").split("(")[0][:28])
              for r in csv.DictReader(open("gpurun_out/prof4q/rc/rc_kernel_trace.csv")))
rows = [r for r in rows if "at::" not in r[2]]
calls, cur = [], []
for r in rows:
    if cur and (r[2].startswith("__amd") and cur[-1][2].startswith("rank_reg")):
        calls.append(cur); cur = []
    cur.append(r)
calls.append(cur)
for c in calls[-14:]:
    t0 = c[0][0]
    print("span %.1f us:" % ((c[-1][1] - t0) / 1e3), " | ".join("%s %.1f" % (n, (e - s) / 1e3) for (s, e, n) in c))
PY
timeout -k 10 300 python scripts/rank_micro.py > gpurun_out/r4q_rank_micro.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4q_rank_micro.log | tail -12
