# Clock and MFMA-busy of the 8-phase GEMM and its epilogue probes at fc500
# (GRBM_GUI_ACTIVE per XCD / kernel duration = shader clock).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p8_clock
for V in 80 93 94; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/p8_clock/v$V -o g -- python3 scripts/gemm_micro.py 3 fc500 $V > gpurun_out/p8_clock/v$V.log 2>&1
  rc=$?
  echo "v$V rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/p8_clock/v$V.log; exit $rc; fi
done
