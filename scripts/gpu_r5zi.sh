# r05 zi: the exact-f32 attention with descriptor loads / stores (no branches) against the conditional form:
# bit-identity tests, then the fp32 tower both ways in one process with kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zi
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "attention_f32" \
  > gpurun_out/r5zi/pytest.log 2>&1 || { tail -30 gpurun_out/r5zi/pytest.log; exit 1; }
tail -2 gpurun_out/r5zi/pytest.log
export F32_VARIANTS=8q,attv1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r5zi/prof -o f32 -- python3 scripts/f32_micro.py 4000 3 > gpurun_out/r5zi/f32_micro.log 2>&1 || { tail -30 gpurun_out/r5zi/f32_micro.log; exit 1; }
grep -v "amdgpu.ids\|simple_timer\|RuntimeWarning\|api.load\|generateRocpd\|tool.cpp" gpurun_out/r5zi/f32_micro.log | tail -4
echo done
