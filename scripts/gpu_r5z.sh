# r05 z: L/14 c_fc in one group per XCD by default -- encode tests, micro, secondary configs on the current tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5z
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5z/pytest_encode.log 2>&1 || { tail -30 gpurun_out/r5z/pytest_encode.log; exit 1; }
tail -2 gpurun_out/r5z/pytest_encode.log
LN_FLAGS=1 timeout -k 10 200 python -u scripts/gemm_micro.py 5 lnfcL 942 > gpurun_out/r5z/lnfcL.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5z/lnfcL.log
timeout -k 10 300 python bench.py --model ViT-B/32 --frames 125000 --queries 32 --steps 2 --warmup 1 --no-cpu-baseline \
  --no-rank-roofline --no-parity-mode > gpurun_out/r5z/config3.log 2> gpurun_out/r5z/config3.err || exit $?
tail -1 gpurun_out/r5z/config3.log | cut -c1-200
timeout -k 10 500 python bench.py --model ViT-L/14 --frames 100000 --queries 256 --steps 1 --warmup 1 --no-cpu-baseline \
  --no-rank-roofline --no-parity-mode > gpurun_out/r5z/config2.log 2> gpurun_out/r5z/config2.err || exit $?
tail -1 gpurun_out/r5z/config2.log | cut -c1-200
timeout -k 10 500 python bench.py --model ViT-L/14@336px --weights fp8 --frames 125000 --queries 1000 --steps 1 --warmup 1 \
  --no-cpu-baseline --no-rank-roofline > gpurun_out/r5z/config4.log 2> gpurun_out/r5z/config4.err || exit $?
tail -1 gpurun_out/r5z/config4.log | cut -c1-200
echo done
