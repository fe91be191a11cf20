# r04 k: where the final entropy pass's time goes: the fused ingest with and without the
# coefficient stores of jp_final (A/B build, MICLIP_JPEG_ABL=1), rocprofv3 kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4k
for a in 0 1; do
  MICLIP_LIB=ab MICLIP_JPEG_ABL=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4k/abl$a -o jpeg -- \
    python3 scripts/jpeg_breakdown.py 8192 fused > gpurun_out/prof4k/abl$a.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob
for a in (0, 1):
    f = glob.glob(f"gpurun_out/prof4k/abl{a}/**/jpeg_kernel_stats.csv", recursive=True)
    if not f:
        f = glob.glob(f"gpurun_out/prof4k/abl{a}/*kernel_stats.csv")
    print("ABL", a, f)
    for r in csv.DictReader(open(f[0])):
        n = r["Name"].replace("void ", "").replace("miclip::(anonymous namespace)::", "").split("(")[0]
        print(f"  {n[:44]:44s} {r['Calls']:>5} {float(r['AverageNs']) / 1e3:9.1f} us")
PY
