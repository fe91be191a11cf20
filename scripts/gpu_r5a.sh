# r05 a: the whole GPU suite (with the new bench-configuration test), then the c_fc / qkv
# A-operand non-temporal and output non-temporal A/B (timing interleaved, then PMC traffic,
# L2 hit rate and MFMA busy per variant)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5a
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5a/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5a/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r5a/pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_config.py -q -s --timeout 200 --timeout-method thread \
  > gpurun_out/r5a/pytest_bench_config.log 2>&1 || exit $?
grep -E "single pass|passed|failed" gpurun_out/r5a/pytest_bench_config.log
export LN_FLAGS=1
timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnfc500 12,76,204,140,44,108 > gpurun_out/r5a/lnfc.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnqkv500 0,64,192 > gpurun_out/r5a/lnqkv.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5a/lnfc.log gpurun_out/r5a/lnqkv.log
for SV in lnfc500:12 lnfc500:76 lnfc500:204 lnqkv500:0 lnqkv500:64; do
  S=${SV%%:*}; V=${SV##*:}; D=gpurun_out/r5a/pmc_${S}_$V
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $D/$c -o run -- \
      python3 scripts/gemm_micro.py 1 $S $V > $D.$c.log 2>&1 || exit $?
  done
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d $D/MFMA -o run -- python3 scripts/gemm_micro.py 1 $S $V > $D.MFMA.log 2>&1 || exit $?
  python3 scripts/pmc_traffic.py $D $S $D/traffic.json || exit $?
done
# the parity mode's kernels (25 % of its step was unattributed)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5a/prof_fp32 -o bench -- \
  python3 bench.py --weights fp32 --steps 2 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-kernel-timing \
  > gpurun_out/r5a/prof_fp32.log 2>&1 || exit $?
echo done
