# A/B of two values of one env switch on the N=1 bench (no tests), alternating:
# usage: VAR=MICLIP_GEMM_VARIANT VA=0 VB=17 bash scripts/gpu_ab_var.sh
mkdir -p gpurun_out
for i in 1 2; do
  for v in $VA $VB; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit $?
    python -c "import json,sys; r=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$VAR=$v', r['value'], r['ms_per_step'], {k:v.get('us') for k,v in r['kernels'].items()})"
  done
done
