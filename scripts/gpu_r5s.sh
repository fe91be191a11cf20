# r05 s: split rank merge for rank_stream (D = 768) too
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5s
timeout -k 10 500 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_rank_scale.py tests/test_gpu_distributed.py \
  tests/test_gpu_service.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5s/pytest_rank.log 2>&1 || { tail -30 gpurun_out/r5s/pytest_rank.log; exit 1; }
tail -2 gpurun_out/r5s/pytest_rank.log
export RANK_MICRO_VARIANTS=default,inl,exact,exact_inl
timeout -k 10 240 python -u scripts/rank_micro.py 5 > gpurun_out/r5s/rank_micro.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5s/rank_micro.log | head -4 | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5s/prof -o rk -- python -u scripts/rank_micro.py 1 > gpurun_out/r5s/prof.log 2>&1 || exit $?
echo done
