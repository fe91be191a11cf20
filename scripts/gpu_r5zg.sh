# r05 zg: fp32 tower split-f16 GEMMs on the 8-phase kernel: F_BEARLY and tile-order groups (A/B), kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zg
export F32_VARIANTS=8q,bearly,ng1,ng3,ab8q
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r5zg/prof -o f32 -- python3 scripts/f32_micro.py 4000 3 > gpurun_out/r5zg/f32_micro.log 2>&1 || { tail -30 gpurun_out/r5zg/f32_micro.log; exit 1; }
grep -v "amdgpu.ids\|simple_timer\|RuntimeWarning\|api.load" gpurun_out/r5zg/f32_micro.log | tail -8
echo done
