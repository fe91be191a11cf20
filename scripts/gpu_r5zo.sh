# r05 zo: the fp32 tower's activation split stored once ([x1 | x2], the 8-phase GEMM's A_DUP read):
# bit-identity (against the ping-pong kernel's full layout), the R@K flow, then the tower both ways
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zo
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py::test_split2h_dedup_layout_bit_identical tests/test_gpu_rk_flow.py \
  tests/test_gpu_ops.py::test_split2h_gemm_8phase_bit_identical tests/test_gpu_ops.py::test_split2h_bit_exact \
  > gpurun_out/r5zo/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r5zo/pytest.log | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
export F32_VARIANTS=8q,nodup
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r5zo/prof -o f32 -- python3 scripts/f32_micro.py 4000 3 > gpurun_out/r5zo/f32_micro.log 2>&1 || { tail -30 gpurun_out/r5zo/f32_micro.log; exit 1; }
grep -v "amdgpu.ids\|simple_timer\|RuntimeWarning\|api.load\|generateRocpd\|tool.cpp" gpurun_out/r5zo/f32_micro.log | tail -4
echo done
