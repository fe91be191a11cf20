# r05 u: MX-fp8 c_fc epilogue with 16-byte e4m3 row stores -- MX tests, micro (fc8), configs[4]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5u
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5u/pytest_mx.log 2>&1 || { tail -30 gpurun_out/r5u/pytest_mx.log; exit 1; }
tail -2 gpurun_out/r5u/pytest_mx.log
MX_MICRO_SHAPES=fc8,fc timeout -k 10 300 python -u scripts/gemm_mx_micro.py 10 > gpurun_out/r5u/mx_micro.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5u/mx_micro.log
echo done
