# r06 y: the fused residual GEMMs (out_proj / c_proj) with the x16 rows' lines warmed into L2
# after the last pair's phase-4 wait (A/B F_WARM, MICLIP_RES_ABL=15) against the product kernel
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6y; mkdir -p $D
RES_VARIANTS=1 timeout -k 10 400 python3 scripts/gemm_micro.py 10 resout500,resproj500 0,6,0,6 > $D/res_warm.log 2>&1 || { tail -20 $D/res_warm.log; exit 1; }
grep -v amdgpu.ids $D/res_warm.log
echo done
