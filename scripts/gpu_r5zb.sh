# r05 zb: where the 8-phase c_fc main loop waits: full / no-MFMA (mode 2) / no-epilogue (mode 4) probes at fc500
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zb
timeout -k 10 300 python -u scripts/gemm_micro.py 5 fc500 110,112,114,110 > gpurun_out/r5zb/fc_abl.log 2>&1 || { cat gpurun_out/r5zb/fc_abl.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5zb/fc_abl.log
echo done
