cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "r32" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_r32_test.log 2>&1
rc=$?; tail -5 gpurun_out/attn_r32_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/attn_micro.py 20 L/14c,L/14@336c > gpurun_out/attn_micro.log 2>&1; rc=$?
cat gpurun_out/attn_micro.log; exit $rc
