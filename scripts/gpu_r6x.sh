# r06 x: the persistent MX-fp8 GEMM with the lean stage loop (compile-time steady waits, per-group
# instantiation, immediate-offset LDS reads) -- MX tests, then the micro against the first form
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6x; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py -q --timeout 300 --timeout-method thread \
  > $D/pytest_mx.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $D/pytest_mx.log | tail -20; exit 1; }
tail -1 $D/pytest_mx.log
timeout -k 10 400 python3 scripts/mx_persist_micro.py 10 fc8,qkv p3:6 > $D/mx_lean.log 2>&1 || { tail -20 $D/mx_lean.log; exit 1; }
timeout -k 10 300 python3 scripts/mx_persist_micro.py 10 out p3:-1 >> $D/mx_lean.log 2>&1 || { tail -20 $D/mx_lean.log; exit 1; }
grep -v amdgpu.ids $D/mx_lean.log
echo done
