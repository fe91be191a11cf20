# parity tests + GEMM microbench + bench (no cpu baseline)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 120 python scripts/gemm_micro.py 20 > gpurun_out/micro.log 2>&1 || exit $?
grep TFLOP gpurun_out/micro.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit $?
python - <<'PY'
import json
r=json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
print(r["value"], r["ms_per_step"], r["config"]["image_chunk"], {k:(v.get("tflops") or v.get("gbs")) for k,v in r["kernels"].items()})
PY
