# r05 zp: which deduplicated split breaks the fp32 tower's bit-identity (A/B mask per producer)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py::test_split2h_dedup_layout_bit_identical > gpurun_out/r5zp/pytest.log 2>&1
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r5zp/pytest.log | tail -8
export F32_VARIANTS=nodup,dup2,8q
timeout -k 10 300 python3 scripts/f32_micro.py 600 1 > gpurun_out/r5zp/f32_micro.log 2>&1 || { tail -30 gpurun_out/r5zp/f32_micro.log; exit 1; }
grep -v "amdgpu.ids\|RuntimeWarning\|api.load" gpurun_out/r5zp/f32_micro.log
echo done
