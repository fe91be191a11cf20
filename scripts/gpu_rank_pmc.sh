# PMC passes over the rank kernel (each pass its own run; counters per the
# MI355X guide's slot limits), plus the counter list for later passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rank_pmc
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rank_pmc/counters_list.txt 2>&1
echo "list rc=$?"
i=0
for C in "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/rank_pmc/p$i -o rank -- python3 scripts/rank_pmc.py 512 5 > gpurun_out/rank_pmc/p$i.log 2>&1
  echo "pass $i ($C) rc=$?"
done
