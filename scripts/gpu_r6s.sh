# r06 s: the fp32 attention on split-f16 operands (attn_f32s_kernel) -- micro, bit identity, fp32 tower tests, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6s; mkdir -p $D
timeout -k 10 300 python3 scripts/attn_f32_micro.py 10000 10 > $D/attn_f32_micro.log 2>&1 || { tail -20 $D/attn_f32_micro.log; exit 1; }
grep -v amdgpu.ids $D/attn_f32_micro.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -k "attention_f32" -s --timeout 200 --timeout-method thread \
  > $D/pytest_attn.log 2>&1 || { grep -E "FAILED|Error|passed|failed|split-f16" $D/pytest_attn.log | tail -30; exit 1; }
tail -1 $D/pytest_attn.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_rk_flow.py tests/test_gpu_flows.py tests/test_gpu_encode.py -q -k "fp32 or f32 or rk" --timeout 300 --timeout-method thread \
  > $D/pytest_fp32.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $D/pytest_fp32.log | tail -20; exit 1; }
tail -1 $D/pytest_fp32.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline > $D/bench.log 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$D/bench.log').read().strip().splitlines()[-1]);p=d['parity_mode'];print('headline',d['value'],'parity',p['value'],p['ms_per_step'],p['kernels']['attention'])"
echo done
