# r05 zr: the fp32 tower with the output split as a compile-time flag: tests (incl. 300 frames against the
# ping-pong full pass), split ops, the tower timing and the bench line with the parity mode
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zr
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rk_flow.py \
  tests/test_gpu_ops.py -k "split2h or attention_f32 or rk_flow or fp32" > gpurun_out/r5zr/pytest.log 2>&1 || { tail -30 gpurun_out/r5zr/pytest.log; exit 1; }
tail -2 gpurun_out/r5zr/pytest.log
F32_VARIANTS=8q,nodup,pp timeout -k 10 400 python3 scripts/f32_micro.py 4000 3 > gpurun_out/r5zr/f32_micro.log 2>&1 || { tail -30 gpurun_out/r5zr/f32_micro.log; exit 1; }
grep -v "amdgpu.ids\|RuntimeWarning\|api.load" gpurun_out/r5zr/f32_micro.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/r5zr/bench.log 2> gpurun_out/r5zr/bench.err || { tail -20 gpurun_out/r5zr/bench.err; exit 1; }
tail -1 gpurun_out/r5zr/bench.log | cut -c1-200
echo done
