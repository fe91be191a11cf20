cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_flows.py tests/test_gpu_service.py -x -q --timeout 150 --timeout-method thread > gpurun_out/rank_test.log 2>&1
rc=$?; tail -4 gpurun_out/rank_test.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_r3h.sh
timeout -k 10 300 python -u scripts/gemm_micro.py 10 fc500,qkv500,out500,proj500 0,125 > gpurun_out/gemm_full.log 2>&1; rc=$?
tail -12 gpurun_out/gemm_full.log; exit $rc
