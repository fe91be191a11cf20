# r04: JPEG final pass with incremental block addressing — tests, ingest timing, per-kernel times
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4g
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4g_pytest.log 2>&1 || exit $?
tail -1 gpurun_out/r4g_pytest.log
timeout -k 10 300 python scripts/jpeg_ingest_micro.py > gpurun_out/r4g_jpeg.log 2>&1 || exit $?
tail -1 gpurun_out/r4g_jpeg.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4g -o jpeg -- \
  python3 scripts/jpeg_breakdown.py 4096 > gpurun_out/prof4g/stdout.log 2>&1 || exit $?
tail -1 gpurun_out/prof4g/stdout.log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof4g/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
