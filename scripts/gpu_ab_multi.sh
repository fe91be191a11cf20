# A/B of several env settings on the N=1 bench, interleaved rounds in one call.
# usage: CONFIGS="A=1;A=2,B=3;..." bash scripts/gpu_ab_multi.sh   (";" separates configs, "," joins vars; "-" = none)
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
IFS=';' read -ra CFG <<< "$CONFIGS"
for i in $(seq 1 $ROUNDS); do
  for c in "${CFG[@]}"; do
    envs=""
    if [ "$c" != "-" ]; then envs=$(echo "$c" | tr ',' ' '); fi
    env $envs timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-rank-roofline ${BENCH_ARGS} > gpurun_out/ab.log 2>&1 || exit $?
    python -c "import json; r=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('[$c]', r['value'], r['ms_per_step'], {k:v.get('us') for k,v in r['kernels'].items() if k.startswith('gemm')})"
  done
done
