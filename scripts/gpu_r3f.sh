# Round 3: attention variants (8x1 / 8x2 / 16x1), rank fold kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -k attention --timeout 120 --timeout-method thread > gpurun_out/r3f_attn_tests.log 2>&1
rc=$?; echo "attention tests rc=$rc"; tail -3 gpurun_out/r3f_attn_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/attn_micro.py 20 "L/14,L/14@336,L/14c,L/14@336c" > gpurun_out/r3f_attn_micro.log 2>&1 || exit $?
cat gpurun_out/r3f_attn_micro.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3f_rprof -o rk -- python3 scripts/rank_fold_trace.py > gpurun_out/r3f_rprof.log 2>&1 || exit $?
cut -d, -f1-4 gpurun_out/r3f_rprof/rk_kernel_stats.csv | sed 's/miclip::(anonymous namespace):://; s/(.*)"/"/' | head -12
