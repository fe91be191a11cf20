# 8-phase GEMM ablation timing at fc500/qkv500 (interleaved, one process) + the
# shader clock of the default and the no-MFMA / no-epilogue probes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p8_abl
timeout -k 10 300 python3 scripts/gemm_micro.py 5 fc500,qkv500 ${VARS:-98,80,91,92,93,94,87,88} > gpurun_out/p8_abl/micro.log 2>&1 || { tail -5 gpurun_out/p8_abl/micro.log; exit 1; }
cat gpurun_out/p8_abl/micro.log
for V in ${CLK:-98 92 94}; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/p8_abl/v$V -o g -- python3 scripts/gemm_micro.py 3 fc500 $V > gpurun_out/p8_abl/v$V.log 2>&1
  rc=$?
  echo "v$V rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/p8_abl/v$V.log; exit $rc; fi
done
