# r06 zb: the rocprofv3 kernel trace of the default bench command itself (20 steps, warmup 5), so the
# per-shape c_fc average comes from the same run as the line's live HIP-event timing
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6zb; mkdir -p $D
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o bench -- \
  python3 bench.py --steps 20 --warmup 5 > $D/bench.log 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
KT=$(find $D/prof -name "*kernel_trace.csv" | head -1)
ST=$(find $D/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/trace_per_shape.py "$KT" $D/r06_zb_bench_per_shape.json "gemm_8q_kernel<7, 0, 942, true> grid=131072: the LN-folded c_fc + QuickGELU at [500000, 3072, 768]"
cp "$ST" $D/r06_zb_bench_kernel_stats.csv
python3 -c "import json;d=json.loads(open('$D/bench.log').read().strip().splitlines()[-1]);r=d['roofline'];print('headline',d['value'],d['ms_per_step'],r['frac'],r['avg_live'] if 'avg_live' in r else r['avg_launch_us'],'parity',d['parity_mode']['value'])"
python3 -c "import json;d=json.load(open('$D/r06_zb_bench_per_shape.json'));print({k:v for k,v in d.items() if 'gemm_8q_kernel<7' in k})"
echo done
