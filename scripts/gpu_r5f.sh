# r05 f: parallel fold_publish + threshold-append slab merge -- rank tests, stamps, micro timings
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5f
timeout -k 10 400 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_rank_scale.py tests/test_gpu_distributed.py \
  tests/test_gpu_service.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5f/pytest_rank.log 2>&1 || { tail -30 gpurun_out/r5f/pytest_rank.log; exit 1; }
tail -2 gpurun_out/r5f/pytest_rank.log
timeout -k 10 120 python -u scripts/rank_stamp.py > gpurun_out/r5f/rank_stamp.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5f/rank_stamp.log
timeout -k 10 180 python -u scripts/rank_micro.py > gpurun_out/r5f/rank_micro.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5f/rank_micro.log | head -4 | cut -c1-220
export LN_FLAGS=1
timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnfc500 430,942 > gpurun_out/r5f/lnfc.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnfc500 430,942 >> gpurun_out/r5f/lnfc.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnqkv500 130,642 > gpurun_out/r5f/lnqkv.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5f/lnfc.log gpurun_out/r5f/lnqkv.log
echo done
