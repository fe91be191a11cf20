# r04 ap: HBM traffic (PMC FETCH_SIZE / WRITE_SIZE, one counter per pass, no trace domains) of the
# product vision-tower GEMMs after the residual fusion and the c_fc epilogue reorder
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc4ap
export GEMM_MICRO_V0=1
SH=lnfc500,lnqkv500,resout500,resproj500
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc4ap/$c -o run -- \
    python3 scripts/gemm_micro.py 1 $SH > gpurun_out/pmc4ap/$c.log 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv \
  -d gpurun_out/pmc4ap/MFMA -o run -- python3 scripts/gemm_micro.py 1 $SH > gpurun_out/pmc4ap/MFMA.log 2>&1 || exit $?
find gpurun_out/pmc4ap -name "*counter_collection.csv" | sort
python3 scripts/pmc_traffic.py gpurun_out/pmc4ap $SH gpurun_out/pmc4ap/r04_zz_gemm_traffic.json
