# PMC of the certified rank pass at 1M x 512 bf16 rows, Q = 32: the default kernel and the
# no-list probe (ABL 3: no scoring MFMAs either): clock, waits, MFMA busy, instruction mix
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cert_pmc
for V in 0 3; do
  i=0
  for C in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"; do
    i=$((i+1))
    MICLIP_RANK_CERT_ABL=$V RC_DT=bf16 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/cert_pmc/v${V}p$i -o c -- python3 scripts/rank_cert_trace.py > gpurun_out/cert_pmc/v${V}p$i.log 2>&1
    rc=$?; echo "v$V pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/cert_pmc/v${V}p$i.log; exit $rc; }
  done
done
