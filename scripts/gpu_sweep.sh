# parity tests, then bench at several image-chunk sizes (kernel timings included)
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for c in ${CHUNKS:-1000}; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --image-chunk $c > gpurun_out/bench_c$c.log 2>&1 || exit $?
  python - "$c" <<'PY'
import json,sys
r=json.loads(open(f"gpurun_out/bench_c{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[1], r["value"], r["ms_per_step"], {k:(v.get("tflops") or v.get("gbs")) for k,v in r["kernels"].items()})
PY
done
