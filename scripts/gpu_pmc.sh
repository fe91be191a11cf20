# PMC counter passes over scripts/gemm_micro.py (each set in its own rocprofv3 run; no trace domains).
# usage: SHAPES_ARG=qkv,long VARIANTS=3 bash scripts/gpu_pmc.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
SH=${SHAPES_ARG:-qkv,long}; VA=${VARIANTS:-3}
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD" \
           "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 scripts/gemm_micro.py 2 $SH $VA > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmc/p$i.log; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc
