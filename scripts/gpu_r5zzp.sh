# r05 zzp: PMC traffic, MFMA busy, clock and L2 hit of the product vision-tower GEMMs on the final binary
# the product vision-tower GEMMs (c_fc / in_proj: whole-line NT stores, early lagging epilogue)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc5zzp
export GEMM_MICRO_V0=1
SH=lnfc500,lnqkv500,resout500,resproj500
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc5zzp/$c -o run -- \
    python3 scripts/gemm_micro.py 1 $SH > gpurun_out/pmc5zzp/$c.log 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d gpurun_out/pmc5zzp/MFMA -o run -- python3 scripts/gemm_micro.py 1 $SH > gpurun_out/pmc5zzp/MFMA.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/pmc5zzp $SH gpurun_out/pmc5zzp/r05_zzp_gemm_traffic.json
echo done
