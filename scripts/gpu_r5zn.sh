# r05 zn: CLS-row last block across chunk boundaries, more 8-phase split-f16 shapes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zn
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_encode.py::test_last_block_cls_rows_across_chunks tests/test_gpu_encode.py::test_last_block_on_cls_rows_bit_identical \
  tests/test_gpu_ops.py::test_split2h_gemm_8phase_bit_identical > gpurun_out/r5zn/pytest.log 2>&1 || { tail -30 gpurun_out/r5zn/pytest.log; exit 1; }
tail -2 gpurun_out/r5zn/pytest.log
echo done
