# r05 b: the fp32 tower on split-f16 GEMMs + the exact-f32 MFMA attention: the new op tests,
# then the whole GPU suite, then the default bench line (parity_mode inside) and a kernel trace
# of the parity mode
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5b
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread \
  -k "split2h or attention_f32" > gpurun_out/r5b/pytest_ops.log 2>&1 || { tail -40 gpurun_out/r5b/pytest_ops.log; exit 1; }
tail -2 gpurun_out/r5b/pytest_ops.log
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5b/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r5b/pytest_gpu.log | tail -30; exit 1; }
tail -2 gpurun_out/r5b/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/r5b/bench.log 2> gpurun_out/r5b/bench.err || { tail -20 gpurun_out/r5b/bench.err; exit 1; }
tail -1 gpurun_out/r5b/bench.log | cut -c1-600
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5b/prof_fp32 -o bench -- \
  python3 bench.py --weights fp32 --steps 2 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-kernel-timing \
  > gpurun_out/r5b/prof_fp32.log 2>&1 || exit $?
export LN_FLAGS=1
timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnfc500 44,46,174 > gpurun_out/r5b/lnfc_full.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnqkv500 0,2,130 > gpurun_out/r5b/lnqkv_full.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5b/lnfc_full.log gpurun_out/r5b/lnqkv_full.log
for SV in lnfc500:174 lnqkv500:130 lnfc500:46; do
  S=${SV%%:*}; V=${SV##*:}; D=gpurun_out/r5b/pmc_${S}_$V
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $D/$c -o run -- \
      python3 scripts/gemm_micro.py 1 $S $V > $D.$c.log 2>&1 || exit $?
  done
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d $D/MFMA -o run -- python3 scripts/gemm_micro.py 1 $S $V > $D.MFMA.log 2>&1 || exit $?
  python3 scripts/pmc_traffic.py $D $S $D/traffic.json || exit $?
done
echo done
