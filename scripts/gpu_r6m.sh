# r06 m: PMC traffic / MFMA busy on the final binary for the secondary configs' dominant kernels
# (configs[2] L/14 c_fc, configs[3] B/32 c_fc at its pass size, configs[4] MX-fp8 c_fc with the
# grouped tile order), then the three secondary bench lines, which read those summaries
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6m
export GEMM_MICRO_V0=1
SH=lnfcL2,lnfc481
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r6m/pmc/$c -o run -- \
    python3 scripts/gemm_micro.py 1 $SH > gpurun_out/r6m/pmc_$c.log 2>&1 || exit $?
done
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d gpurun_out/r6m/pmc/MFMA -o run -- python3 scripts/gemm_micro.py 1 $SH > gpurun_out/r6m/pmc_MFMA.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/r6m/pmc $SH profiles/r06_m_gemm_traffic.json
unset GEMM_MICRO_V0
TAG=r06_m bash scripts/gpu_fp8_traffic.sh > gpurun_out/r6m/fp8_traffic.log 2>&1 || { tail -20 gpurun_out/r6m/fp8_traffic.log; exit 1; }
cp gpurun_out/r06_m_fp8_gemm_traffic.json profiles/
tail -1 gpurun_out/r6m/fp8_traffic.log | cut -c1-300
bash scripts/gpu_r6g.sh > gpurun_out/r6m/configs.log 2>&1 || { tail -20 gpurun_out/r6m/configs.log; exit 1; }
cp gpurun_out/r6g/config2.log gpurun_out/r6m/config2.json; cp gpurun_out/r6g/config3.log gpurun_out/r6m/config3.json; cp gpurun_out/r6g/config4.log gpurun_out/r6m/config4.json
tail -4 gpurun_out/r6m/configs.log | cut -c1-200
echo done
