# r06 t: the fp32 attention writing out_proj's split operand (attention_f32_split) -- the attention
# tests first, then the whole GPU suite, smoke and the bench line (parity mode)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6t; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -k "attention_f32" -s --timeout 200 --timeout-method thread \
  > $D/pytest_attn.log 2>&1 || { grep -E "FAILED|Error|passed|failed|split-f16" $D/pytest_attn.log | tail -30; exit 1; }
tail -1 $D/pytest_attn.log
timeout -k 10 300 python3 scripts/attn_f32_micro.py 10000 10 > $D/attn_f32_micro.log 2>&1 || { tail -20 $D/attn_f32_micro.log; exit 1; }
grep -v amdgpu.ids $D/attn_f32_micro.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread \
  > $D/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $D/pytest_gpu.log | tail -30; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $D/bench.log 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$D/bench.log').read().strip().splitlines()[-1]);p=d['parity_mode'];print('headline',d['value'],d['roofline']['frac'],'parity',p['value'],p['ms_per_step'],p['kernels']['attention'])"
echo done
