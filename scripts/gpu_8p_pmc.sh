# PMC passes over the 8-phase GEMM (v80) and its no-DMA probe (v91) at qkv500:
# clock (GRBM), MFMA busy, LDS bank conflicts, wait cycles.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p8_pmc
for V in 80 91; do
  i=0
  for C in "GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM TA_TA_BUSY_sum FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/p8_pmc/v${V}_p$i -o g -- python3 scripts/gemm_micro.py 2 qkv500 $V > gpurun_out/p8_pmc/v${V}_p$i.log 2>&1
    rc=$?
    echo "v$V pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/p8_pmc/v${V}_p$i.log; exit $rc; fi
  done
done
