# PMC traffic + MFMA busy of the MX-fp8 c_fc GEMM (configs[4]), one counter group per pass
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-rXX}
mkdir -p gpurun_out/fp8prof
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/fp8prof/$c -o run -- \
    python3 scripts/fp8_traffic.py run > gpurun_out/fp8prof/$c.log 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/fp8prof/MFMA -o run -- python3 scripts/fp8_traffic.py run > gpurun_out/fp8prof/MFMA.log 2>&1 || exit $?
python3 scripts/fp8_traffic.py summarize gpurun_out/fp8prof gpurun_out/${TAG}_fp8_gemm_traffic.json
