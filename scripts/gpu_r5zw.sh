# r05 zw: kernel stats of the fp32 tower (parity mode) on the final tree, 10k frames
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zw
F32_VARIANTS=8q timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5zw/prof -o f32 -- python3 scripts/f32_micro.py 10000 1 > gpurun_out/r5zw/f32.log 2>&1 || { tail -20 gpurun_out/r5zw/f32.log; exit 1; }
grep -v "amdgpu.ids\|RuntimeWarning\|api.load\|simple_timer\|generateRocpd\|tool.cpp" gpurun_out/r5zw/f32.log | tail -4
echo done
