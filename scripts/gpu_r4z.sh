# r04 z: per-block window masks (no coefficient memset; the IDCT reads written windows only): JPEG parity tests, then the
# fused ingest's kernel stats and the ingest rate
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4z
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_realframes.py tests/test_gpu_service.py -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/r4z_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4z_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4z -o jpeg -- \
  python3 scripts/jpeg_breakdown.py 8192 fused > gpurun_out/prof4z/breakdown.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof4z/jpeg_kernel_stats.csv")):
    n = r["Name"].replace("void ", "").replace("miclip::(anonymous namespace)::", "").split("(")[0]
    print(f"  {n[:44]:44s} {r['Calls']:>5} {float(r['AverageNs']) / 1e3:9.1f} us")
PY
timeout -k 10 300 python scripts/jpeg_ingest_micro.py > gpurun_out/r4z_jpeg.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4z_jpeg.log
