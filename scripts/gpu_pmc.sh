# GEMM microbench + PMC counter passes (each counter set in its own rocprofv3 run; no trace domains)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
timeout -k 10 120 python scripts/gemm_micro.py 20 > gpurun_out/pmc/micro.log 2>&1 || exit $?
cat gpurun_out/pmc/micro.log
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 scripts/gemm_micro.py 3 ${SHAPES_ARG:-fc,proj,sq4096} > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; }
done
ls -R gpurun_out/pmc | head -40
