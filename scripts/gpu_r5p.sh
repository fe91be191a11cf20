# r05 p: split rank merge (tests + micro A/B + trace) and the deferred-epilogue c_fc kernel (gemm_1d) A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5p
export LN_FLAGS=1
timeout -k 10 120 python -u scripts/gemm_micro.py 3 lnfc1k 942,1000 > gpurun_out/r5p/lnfc_small.log 2>&1 || { cat gpurun_out/r5p/lnfc_small.log; exit 1; }
timeout -k 10 120 python -u scripts/gemm_micro.py 3 lnfc40k 942,1000 >> gpurun_out/r5p/lnfc_small.log 2>&1 || { cat gpurun_out/r5p/lnfc_small.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5p/lnfc_small.log
timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnfc500 942,1000,1004 > gpurun_out/r5p/lnfc.log 2>&1 || { cat gpurun_out/r5p/lnfc.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5p/lnfc.log
unset LN_FLAGS
timeout -k 10 500 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_rank_scale.py tests/test_gpu_distributed.py \
  tests/test_gpu_service.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5p/pytest_rank.log 2>&1 || { tail -30 gpurun_out/r5p/pytest_rank.log; exit 1; }
tail -2 gpurun_out/r5p/pytest_rank.log
export RANK_MICRO_VARIANTS=default,inl,exact,exact_inl
timeout -k 10 240 python -u scripts/rank_micro.py 5 > gpurun_out/r5p/rank_micro.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5p/rank_micro.log | head -4 | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5p/prof -o rk -- python -u scripts/rank_micro.py 1 > gpurun_out/r5p/prof.log 2>&1 || exit $?
echo done
