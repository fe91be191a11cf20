# 8q kernel: bit-identity tests vs the 8p kernel, then interleaved timing at the bench shapes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p8q
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x -k "8phase or test_gemm" --timeout 120 --timeout-method thread > gpurun_out/p8q/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/p8q/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/gemm_micro.py 5 ${SHAPES:-fc500,qkv500,out500,proj500} ${VARS:-98,110,111,112,114,94} > gpurun_out/p8q/micro.log 2>&1 || { tail -5 gpurun_out/p8q/micro.log; exit 1; }
cat gpurun_out/p8q/micro.log
