# A/B of an env switch on the N=1 bench: gpu tests first, then the bench with
# VAR=0 and VAR=1 alternating (usage: VAR=MICLIP_RESID16 bash scripts/gpu_ab_env.sh)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
for i in 1 2; do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit $?
    python -c "import json,sys; r=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$VAR=$v', r['value'], r['ms_per_step'], {k:v.get('us') for k,v in r['kernels'].items()})"
  done
done
