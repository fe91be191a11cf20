# PMC of the default rank kernel at 1M x 512 f32, Q = 32: clock, MFMA busy, waits, FETCH
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rank_pmc2
i=0
for C in "FETCH_SIZE" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/rank_pmc2/p$i -o rank -- python3 scripts/rank_pmc.py 512 5 ${VARENV} > gpurun_out/rank_pmc2/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
