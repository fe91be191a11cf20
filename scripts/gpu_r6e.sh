# r06 e: the final-binary evidence for the bench line: rocprofv3 kernel trace of bench.py (per shape),
# PMC traffic / MFMA busy of the product vision GEMMs, and the vendor library (hipBLASLt) at the
# bench's 500k-row shapes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6e
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6e/prof -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/r6e/prof.log 2>&1 || { tail -20 gpurun_out/r6e/prof.log; exit 1; }
KT=$(find gpurun_out/r6e/prof -name "*kernel_trace.csv" | head -1)
ST=$(find gpurun_out/r6e/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/trace_per_shape.py "$KT" gpurun_out/r6e/r06_e_bench_per_shape.json "gemm_8q_kernel<7, 0, 942, true> grid=131072: the LN-folded c_fc + QuickGELU at [500000, 3072, 768]"
cp "$ST" gpurun_out/r6e/r06_e_bench_kernel_stats.csv
export GEMM_MICRO_V0=1
SH=lnfc500,lnqkv500,resout500,resproj500
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r6e/pmc/$c -o run -- \
    python3 scripts/gemm_micro.py 1 $SH > gpurun_out/r6e/pmc_$c.log 2>&1 || exit $?
done
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d gpurun_out/r6e/pmc/MFMA -o run -- python3 scripts/gemm_micro.py 1 $SH > gpurun_out/r6e/pmc_MFMA.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/r6e/pmc $SH gpurun_out/r6e/r06_e_gemm_traffic.json
timeout -k 10 300 python3 scripts/blas_ref.py 10 > gpurun_out/r6e/hipblaslt.log 2>&1 || { tail -5 gpurun_out/r6e/hipblaslt.log; exit 1; }
grep hipblaslt gpurun_out/r6e/hipblaslt.log
echo done
