# r04 ak: persistent short-attention A/B micro, then the full check of the product tree (every GPU
# test, smoke, JPEG ingest, the default bench line, kernel trace of the bench)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4ak
timeout -k 10 300 python -u scripts/attn_micro.py 10 B/32c > gpurun_out/r4ak_attn.log 2>&1 || exit $?
cat gpurun_out/r4ak_attn.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread > gpurun_out/r4ak_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r4ak_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ak_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r4ak_smoke.log
timeout -k 10 300 python scripts/jpeg_ingest_micro.py > gpurun_out/r4ak_jpeg.log 2>&1 || exit $?
tail -1 gpurun_out/r4ak_jpeg.log
timeout -k 10 700 python bench.py --steps 20 --warmup 3 > gpurun_out/r4ak_bench.log 2> gpurun_out/r4ak_bench.err || exit $?
tail -1 gpurun_out/r4ak_bench.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4ak -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/prof4ak/stdout.log 2>&1 || exit $?
echo done
