# rocprofv3 kernel trace of the bench + HBM traffic (FETCH_SIZE / WRITE_SIZE, one
# counter set per pass, no trace domains) of the dominant GEMM at the bench shape
# + the hipBLASLt bar.  Outputs under gpurun_out/prof.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_stdout.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/prof/$c -o run -- \
    python3 scripts/gemm_micro.py 1 ${SHAPES_ARG:-fc250,qkv250,out250,proj250} > gpurun_out/prof/$c.log 2>&1 || exit $?
done
timeout -k 10 120 python3 scripts/blas_ref.py > gpurun_out/prof/blas.log 2>&1 || exit $?
cat gpurun_out/prof/blas.log
find gpurun_out/prof -name "*.csv" | head -20
