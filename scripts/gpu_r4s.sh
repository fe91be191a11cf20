# r04 s: double-buffered fp32 GEMM (parity mode): parity tests (operator, fp32 towers, R@K flow), timing
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py -k gemm_f32 tests/test_gpu_rk_flow.py tests/test_gpu_encode.py tests/test_gpu_flows.py -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/r4s_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4s_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/gemm_f32_micro.py > gpurun_out/r4s_gemm_f32.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4s_gemm_f32.log
