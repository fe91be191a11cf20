# r05 zf: kernel stats of the fp32 tower, 8-phase split-f16 GEMMs against the ping-pong ones (one process),
# and the rk-flow / fp32-tower tests in full
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zf
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_rk_flow.py > gpurun_out/r5zf/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r5zf/pytest.log; exit 1; }
tail -3 gpurun_out/r5zf/pytest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5zf/prof -o f32 -- python3 scripts/f32_micro.py 10000 1 > gpurun_out/r5zf/f32_prof.log 2>&1 || { tail -20 gpurun_out/r5zf/f32_prof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5zf/f32_prof.log | tail -4
find gpurun_out/r5zf/prof -name "*stats*"
echo done
