# r05 j: fused out_proj / c_proj with the lagging group's epilogue early (F_BEARLY, v9): bit
# identity, then interleaved timing
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5j
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -q -k "residual" --timeout 120 --timeout-method thread \
  > gpurun_out/r5j/pytest_res.log 2>&1 || { tail -30 gpurun_out/r5j/pytest_res.log; exit 1; }
tail -1 gpurun_out/r5j/pytest_res.log
RES_VARIANTS=1 timeout -k 10 300 python -u scripts/gemm_micro.py 10 resout500,resproj500 0,9,0,9 > gpurun_out/r5j/res_bearly.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5j/res_bearly.log
echo done
