# r06 b: config-scale + whole GPU suite, smoke, bench line; then a FETCH sweep of the LN-folded
# c_fc / in_proj over M (does the A re-fetch grow with the pass length? -- CU drift hypothesis)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6b
# the per-XCD claimed tile order (F_DYN, A/B) against the product c_fc / in_proj: timing + maxdiff,
# then its FETCH / WRITE
LN_FLAGS=1 timeout -k 10 180 python3 scripts/gemm_micro.py 20 lnfc500,lnqkv500 0,10000 > gpurun_out/r6b/dyn_micro.log 2>&1 || { tail -20 gpurun_out/r6b/dyn_micro.log; exit 1; }
cat gpurun_out/r6b/dyn_micro.log | grep -v amdgpu.ids
for c in FETCH_SIZE WRITE_SIZE; do
  GEMM_MICRO_V0=1 MICLIP_8Q_DYN=1 timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r6b/pmcdyn/$c -o run -- \
    python3 scripts/gemm_micro.py 1 lnfc500,lnqkv500 > gpurun_out/r6b/pmcdyn_$c.log 2>&1 || exit $?
done
GEMM_MICRO_V0=1 MICLIP_8Q_DYN=1 timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d gpurun_out/r6b/pmcdyn/MFMA -o run -- python3 scripts/gemm_micro.py 1 lnfc500,lnqkv500 > gpurun_out/r6b/pmcdyn_MFMA.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/r6b/pmcdyn lnfc500,lnqkv500 gpurun_out/r6b/r06_b_gemm_traffic_dyn.json
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread \
  > gpurun_out/r6b/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r6b/pytest_gpu.log | tail -30; exit 1; }
tail -2 gpurun_out/r6b/pytest_gpu.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r6b/smoke.log 2>&1 || { tail -20 gpurun_out/r6b/smoke.log; exit 1; }
tail -1 gpurun_out/r6b/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/r6b/bench.log 2> gpurun_out/r6b/bench.err || { tail -20 gpurun_out/r6b/bench.err; exit 1; }
tail -1 gpurun_out/r6b/bench.log | cut -c1-800
export GEMM_MICRO_V0=1
SH=lnfc40k,lnfc100,lnfc250,lnfc500,lnqkv100,lnqkv250,lnqkv500
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r6b/pmc/$c -o run -- \
    python3 scripts/gemm_micro.py 1 $SH > gpurun_out/r6b/pmc_$c.log 2>&1 || exit $?
done
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d gpurun_out/r6b/pmc/MFMA -o run -- python3 scripts/gemm_micro.py 1 $SH > gpurun_out/r6b/pmc_MFMA.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/r6b/pmc $SH gpurun_out/r6b/r06_b_gemm_traffic_mscale.json
echo done
