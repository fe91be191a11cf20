# A/B of two bench argument sets on the N=1 bench (no tests), alternating:
# usage: A="--image-chunk 5000" B="--image-chunk 5242" bash scripts/gpu_ab_args.sh
mkdir -p gpurun_out
for i in 1 2; do
  for v in A B; do
    timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${!v} > gpurun_out/ab_$v.log 2>&1 || exit $?
    python -c "import json,sys; r=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$v', '${!v}', r['value'], r['ms_per_step'], {k:v.get('us') for k,v in r['kernels'].items()})"
  done
done
