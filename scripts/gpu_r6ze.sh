# r06 ze: the fp32 attention's split output with the bound reduced late (A/B) against the product
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6ze; mkdir -p $D
timeout -k 10 300 python3 scripts/attn_split_micro.py 10000 10 > $D/attn_split_micro.log 2>&1 || { tail -20 $D/attn_split_micro.log; exit 1; }
grep -v amdgpu.ids $D/attn_split_micro.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -k "attention_f32_split" --timeout 200 --timeout-method thread \
  > $D/pytest_attn.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $D/pytest_attn.log | tail -20; exit 1; }
tail -1 $D/pytest_attn.log
echo done
