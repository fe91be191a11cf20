# r06 zc: the fp32 attention split output with the bound row-max load issued first and reduced at the first block's stores
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6zc; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -k "attention_f32" --timeout 200 --timeout-method thread \
  > $D/pytest_attn.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $D/pytest_attn.log | tail -20; exit 1; }
tail -1 $D/pytest_attn.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_rk_flow.py tests/test_gpu_flows.py tests/test_gpu_encode.py -q -k "fp32 or f32 or rk" --timeout 300 --timeout-method thread \
  > $D/pytest_fp32.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $D/pytest_fp32.log | tail -20; exit 1; }
tail -1 $D/pytest_fp32.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline > $D/bench.log 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$D/bench.log').read().strip().splitlines()[-1]);p=d['parity_mode'];print('headline',d['value'],'parity',p['value'],p['ms_per_step'],p['kernels']['attention'],p['kernels']['attention_split'])"
echo done
