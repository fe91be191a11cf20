# r04: vectorised fused JPEG transform + attention A/B variants: tests, ingest timing, kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4e
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_ops.py -x -q -rf --timeout 200 \
  --timeout-method thread > gpurun_out/r4e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4e_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/jpeg_ingest_micro.py > gpurun_out/r4e_jpeg.log 2>&1 || exit $?
tail -1 gpurun_out/r4e_jpeg.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4e -o jpeg -- \
  python3 scripts/jpeg_ingest_micro.py 4096 > gpurun_out/prof4e/stdout.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof4e/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
