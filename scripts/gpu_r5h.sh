# r05 h: the fused out_proj / c_proj with a start stagger (x16 read bursts spread); the whole GPU
# suite (the fp32 tower's fused c_fc split, the kernel-event timing); the bench line with the live
# c_fc timing and the parity mode
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5h
RES_VARIANTS=1 timeout -k 10 300 python -u scripts/gemm_micro.py 10 resout500,resproj500 0,6,7,8,0 > gpurun_out/r5h/res_stagger.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5h/res_stagger.log
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5h/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r5h/pytest_gpu.log | tail -30; exit 1; }
tail -2 gpurun_out/r5h/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-rank-roofline > gpurun_out/r5h/bench.log 2> gpurun_out/r5h/bench.err || { tail -20 gpurun_out/r5h/bench.err; exit 1; }
tail -1 gpurun_out/r5h/bench.log | cut -c1-300
echo done
