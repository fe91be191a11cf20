# r06 zd: sanity of the final tree's libraries (smoke, the fp32 attention and MX tests)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6zd; mkdir -p $D
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_mx.py -q -k "attention_f32 or mx or small_tiles" --timeout 300 --timeout-method thread \
  > $D/pytest.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $D/pytest.log | tail -20; exit 1; }
tail -1 $D/pytest.log
echo done
