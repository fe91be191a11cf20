# r06 f: which hipBLASLt kernels run the 500k-row bf16 GEMMs (macro tile, MFMA, depth-U from the names)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6f
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6f/prof -o blas -- \
  python3 scripts/blas_ref.py 3 > gpurun_out/r6f/blas.log 2>&1 || { tail -20 gpurun_out/r6f/blas.log; exit 1; }
ST=$(find gpurun_out/r6f/prof -name "*kernel_stats.csv" | head -1)
cp "$ST" gpurun_out/r6f/r06_f_hipblaslt_kernel_stats.csv
cut -c1-400 gpurun_out/r6f/r06_f_hipblaslt_kernel_stats.csv | head -20
echo done
