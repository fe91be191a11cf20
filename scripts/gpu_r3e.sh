# Round 3: attention two tiles per wave, rank_reg for 16-bit corpora, JPEG v3 ingest (native gather, pipelined launches).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -k attention --timeout 120 --timeout-method thread > gpurun_out/r3e_attn_tests.log 2>&1
rc=$?; echo "attention tests rc=$rc"; tail -3 gpurun_out/r3e_attn_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_rank.py -q --timeout 120 --timeout-method thread > gpurun_out/r3e_rank_tests.log 2>&1
rc=$?; echo "rank tests rc=$rc"; tail -3 gpurun_out/r3e_rank_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/rank_micro.py 2 > gpurun_out/r3e_rank_micro.log 2>&1 || exit $?
grep -v "^{" gpurun_out/r3e_rank_micro.log
timeout -k 10 300 python scripts/attn_micro.py 20 > gpurun_out/r3e_attn_micro.log 2>&1 || exit $?
cat gpurun_out/r3e_attn_micro.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_service.py tests/test_gpu_flows.py -q --timeout 300 --timeout-method thread > gpurun_out/r3e_jpeg_tests.log 2>&1
rc=$?; echo "jpeg tests rc=$rc"; tail -5 gpurun_out/r3e_jpeg_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python scripts/jpeg_breakdown.py 8192 > gpurun_out/r3e_breakdown.log 2>&1 || exit $?
cat gpurun_out/r3e_breakdown.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3e_jprof -o jp -- python3 scripts/jpeg_micro.py 8192 > gpurun_out/r3e_jprof.log 2>&1 || exit $?
tail -2 gpurun_out/r3e_jprof.log
cut -d, -f1-4 gpurun_out/r3e_jprof/jp_kernel_stats.csv | sed 's/miclip::(anonymous namespace):://; s/(.*)"/"/' | head -16
