# r06 n: the fp32 tower's attention with every load ahead of the first MFMA -- bit identity, the
# micro at 10k frames, the fp32 tower tests, then the parity mode through the bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6n
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -k "attention_f32" --timeout 200 --timeout-method thread \
  > gpurun_out/r6n/pytest_attn.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r6n/pytest_attn.log | tail -20; exit 1; }
tail -1 gpurun_out/r6n/pytest_attn.log
timeout -k 10 300 python3 scripts/attn_f32_micro.py 10000 10 > gpurun_out/r6n/attn_f32_micro.log 2>&1 || { tail -20 gpurun_out/r6n/attn_f32_micro.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6n/attn_f32_micro.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_rk_flow.py tests/test_gpu_flows.py tests/test_gpu_encode.py -q -k "fp32 or f32 or rk" --timeout 300 --timeout-method thread \
  > gpurun_out/r6n/pytest_fp32.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r6n/pytest_fp32.log | tail -20; exit 1; }
tail -1 gpurun_out/r6n/pytest_fp32.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline > gpurun_out/r6n/bench.log 2> gpurun_out/r6n/bench.err || { tail -20 gpurun_out/r6n/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6n/bench.log').read().strip().splitlines()[-1]);p=d['parity_mode'];print('headline',d['value'],'parity',p['value'],p['ms_per_step'],p['kernels']['attention'])"
echo done
