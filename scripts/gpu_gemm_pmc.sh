# PMC passes over the persistent GEMM at fc500 for two tile orders
# (v40 = m-major, v44 = n-groups of 4) and the loads-only probe (v33).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gemm_pmc
for V in 40 44 33; do
  i=0
  for C in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE GRBM_COUNT TA_TA_BUSY_sum TA_BUFFER_READ_LDS_WAVEFRONTS_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/gemm_pmc/v${V}_p$i -o g -- python3 scripts/gemm_micro.py 2 fc500 $V > gpurun_out/gemm_pmc/v${V}_p$i.log 2>&1
    echo "v$V pass $i rc=$?"
  done
done
