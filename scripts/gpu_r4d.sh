# r04: attention split-last-tile tests + micro, then the bench line and kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4d
true || timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_encode.py -x -q -rf --timeout 200 \
  --timeout-method thread > gpurun_out/r4d_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4d_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
ATTN_VARS=11,12 timeout -k 10 300 python scripts/attn_micro.py 20 L/14c,L/14 > gpurun_out/r4d_attn.log 2>&1 || exit $?
cat gpurun_out/r4d_attn.log | grep -v amdgpu.ids
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-parity-mode > gpurun_out/r4d_bench.log 2> gpurun_out/r4d_bench.err || exit $?
tail -1 gpurun_out/r4d_bench.log | cut -c1-300
tail -1 gpurun_out/r4d_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['kernels']['jpeg_ingest_720p'])); print(d['roofline']['avg_launch_us'], d['kernels']['gemm_qkv'], d['kernels']['gemm_fc'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4d -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/prof4d/stdout.log 2>&1 || exit $?
find gpurun_out/prof4d -name "*kernel_stats.csv" | head -2
