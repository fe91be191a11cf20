# r04 p: transform with 24-bit multiplies and row-fastest H pass: JPEG parity tests, then the
# fused ingest's kernel stats and the ingest rate
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4p
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_realframes.py tests/test_gpu_service.py -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/r4p_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4p_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4p -o jpeg -- \
  python3 scripts/jpeg_breakdown.py 8192 fused > gpurun_out/prof4p/breakdown.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof4p/jpeg_kernel_stats.csv")):
    n = r["Name"].replace("void ", "").replace("miclip::(anonymous namespace)::", "").split("(")[0]
    print(f"  {n[:44]:44s} {r['Calls']:>5} {float(r['AverageNs']) / 1e3:9.1f} us")
PY
timeout -k 10 300 python scripts/jpeg_ingest_micro.py > gpurun_out/r4p_jpeg.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4p_jpeg.log
# the certified rank call's kernels and the gaps between them (1M x 512, f32 then bf16)
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof4p/rc -o rc -- python3 scripts/rank_cert_trace.py > gpurun_out/prof4p/rc.log 2>&1 || exit $?
python3 - <<'PY'
import csv
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("void ", "").replace("miclip::(anonymous namespace)::", "").split("(")[0][:40])
              for r in csv.DictReader(open("gpurun_out/prof4p/rc/rc_kernel_trace.csv")))
rows = [r for r in rows if "rank" in r[2] or "fill" in r[2] or "cert" in r[2] or "rescore" in r[2]]
# the last 3 calls of each dtype: print each kernel's duration and the gap before it
calls, cur = [], []
for r in rows:
    if cur and r[0] - cur[-1][1] > 200000:   # > 200 us idle: a new call
        calls.append(cur); cur = []
    cur.append(r)
calls.append(cur)
for c in calls[7:10] + calls[17:20]:
    t0 = c[0][0]
    print("call span %.1f us" % ((c[-1][1] - t0) / 1e3), " | ".join("%s %.1f (+%.1f)" % (n, (e - s) / 1e3, (s - (c[i - 1][1] if i else s)) / 1e3) for i, (s, e, n) in enumerate(c)))
PY
