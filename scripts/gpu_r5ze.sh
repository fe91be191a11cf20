# r05 ze: the fp32 tower's split-f16 GEMMs on the 8-phase kernel (gemm_8q SPL epilogues):
# bit-identity against the ping-pong kernel, then the parity mode's tower time, both libraries
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5ze
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ops.py -k "split2h" tests/test_gpu_rk_flow.py > gpurun_out/r5ze/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r5ze/pytest.log; exit 1; }
tail -3 gpurun_out/r5ze/pytest.log
timeout -k 10 400 python -u scripts/f32_micro.py 2000 3 > gpurun_out/r5ze/f32_micro_2k.log 2>&1 || { cat gpurun_out/r5ze/f32_micro_2k.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5ze/f32_micro_2k.log
timeout -k 10 400 python -u scripts/f32_micro.py 10000 3 > gpurun_out/r5ze/f32_micro_10k.log 2>&1 || { cat gpurun_out/r5ze/f32_micro_10k.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5ze/f32_micro_10k.log
echo done
