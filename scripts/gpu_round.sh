# Round check on one GPU: every GPU test, smoke, PMC traffic (FETCH_SIZE / WRITE_SIZE
# passes) and MFMA busy (GRBM + SQ pass) of the four bench GEMMs, written to profiles/
# on the box so the bench line picks them up, the bench line, and a rocprofv3 kernel
# trace of the bench.
# usage: TAG=r02_v2 bash scripts/gpu_round.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-rXX}
mkdir -p gpurun_out/prof
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/prof/$c -o run -- \
    python3 scripts/gemm_micro.py 1 fc500,qkv500,out500,proj500 > gpurun_out/prof/$c.log 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/prof/MFMA -o run -- \
  python3 scripts/gemm_micro.py 1 fc500,qkv500,out500,proj500 > gpurun_out/prof/MFMA.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/prof fc500,qkv500,out500,proj500 gpurun_out/${TAG}_gemm_traffic.json || exit $?
cp gpurun_out/${TAG}_gemm_traffic.json profiles/
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 3} > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log > gpurun_out/${TAG}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline > gpurun_out/prof/bench_stdout.log 2>&1 || exit $?
cat gpurun_out/${TAG}_bench.json
