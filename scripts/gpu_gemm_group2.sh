# gemm_8q default grouped order (c_fc) vs forced raster (131): GEMM tests, micro, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/grp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_encode.py -q -x --timeout 120 --timeout-method thread > gpurun_out/grp/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/grp/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/gemm_micro.py 10 fc500,qkv500 0,131,136 > gpurun_out/grp/micro2.log 2>&1 || exit $?
cat gpurun_out/grp/micro2.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-rank-roofline > gpurun_out/grp/bench.log 2>&1 || exit $?
tail -1 gpurun_out/grp/bench.log | cut -c1-400
