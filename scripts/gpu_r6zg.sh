# r06 zg: the whole GPU suite on the final tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6zg; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread \
  > $D/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $D/pytest_gpu.log | tail -30; exit 1; }
tail -2 $D/pytest_gpu.log
echo done
