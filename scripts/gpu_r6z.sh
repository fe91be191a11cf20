# r06 z: the final round-6 tree -- the whole GPU suite, smoke, the bench line, the rocprofv3 kernel
# trace of the bench (per shape) and the three secondary configs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6z; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread \
  > $D/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $D/pytest_gpu.log | tail -30; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $D/bench.log 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$D/bench.log').read().strip().splitlines()[-1]);p=d['parity_mode'];print('headline',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['achieved'],'parity',p['value'],p['ms_per_step'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
KT=$(find $D/prof -name "*kernel_trace.csv" | head -1)
ST=$(find $D/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/trace_per_shape.py "$KT" $D/r06_z_bench_per_shape.json "gemm_8q_kernel<7, 0, 942, true> grid=131072: the LN-folded c_fc + QuickGELU at [500000, 3072, 768]"
cp "$ST" $D/r06_z_bench_kernel_stats.csv
tail -1 $D/prof.log | cut -c1-300
bash scripts/gpu_r6g.sh > $D/configs.log 2>&1 || { tail -20 $D/configs.log; exit 1; }
cp gpurun_out/r6g/config2.log $D/config2.json; cp gpurun_out/r6g/config3.log $D/config3.json; cp gpurun_out/r6g/config4.log $D/config4.json
tail -4 $D/configs.log | cut -c1-200
echo done
