cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_ops.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r3j_test.log 2>&1
rc=$?; tail -3 gpurun_out/r3j_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/rank_micro.py 3 > gpurun_out/rank_micro.log 2>&1; rc=$?
head -4 gpurun_out/rank_micro.log; exit $rc
