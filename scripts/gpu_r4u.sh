# r04 u: fp32 tower on split-bf16 GEMMs (mi_op_split6 tests, parity-mode timing): its parity tests (fp32 towers vs fp64 / HF goldens,
# the R@K flow bit-identity, configs[0] flow, operator GEMM), then the parity-mode rate
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1100 python -u -m pytest tests/test_gpu_rk_flow.py tests/test_gpu_encode.py tests/test_gpu_flows.py tests/test_gpu_ops.py -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/r4u_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4u_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-rank-roofline > gpurun_out/r4u_bench.log 2> gpurun_out/r4u_bench.err || exit $?
python3 -c "
import json; d = json.loads(open('gpurun_out/r4u_bench.log').read().strip().splitlines()[-1])
print(d['value'], json.dumps(d['parity_mode']))"
