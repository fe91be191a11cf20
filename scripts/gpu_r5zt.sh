# r05 zt: the SPL epilogue without its runtime bias branch (bias-less calls on the ping-pong kernel): split / fp32 tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zt
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rk_flow.py \
  tests/test_gpu_ops.py -k "split2h or attention_f32 or rk_flow or fp32" > gpurun_out/r5zt/pytest.log 2>&1 || { tail -30 gpurun_out/r5zt/pytest.log; exit 1; }
tail -2 gpurun_out/r5zt/pytest.log
F32_NO_EXIT=1 F32_VARIANTS=pp,8q,nodup timeout -k 10 400 python3 scripts/f32_micro.py 4000 3 > gpurun_out/r5zt/f32_micro.log 2>&1 || { tail -30 gpurun_out/r5zt/f32_micro.log; exit 1; }
grep -v "amdgpu.ids\|RuntimeWarning\|api.load" gpurun_out/r5zt/f32_micro.log
echo done
