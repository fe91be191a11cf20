# r04 first GPU pass: the fp16-corpus parity tests, the config-scale rank-vs-oracle tests,
# the JPEG segment-contract test, the rank/jpeg/service suites, then one bench line
# (with the fp32 parity-mode measurement).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_rank_scale.py tests/test_gpu_service.py \
  tests/test_gpu_jpeg.py -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/r4a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r4a_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r4a_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r4a_bench.log
