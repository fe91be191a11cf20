# r04 i: operator parity of the LayerNorm-folded GEMM / residual_stats, their timing at the
# bench shape, PMC traffic + MFMA busy of the folded GEMMs (profiles/r04_i_gemm_traffic.json,
# read by the bench line), the bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4i
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "gemm_ln or residual_stats" -q -rf --timeout 120 --timeout-method thread > gpurun_out/r4i_pytest.log 2>&1 || exit $?
tail -2 gpurun_out/r4i_pytest.log
timeout -k 10 300 python scripts/gemm_micro.py 20 lnfc500,fc500,lnqkv500,qkv500 > gpurun_out/r4i_gemm_micro.log 2>&1 || exit $?
cat gpurun_out/r4i_gemm_micro.log | grep -v amdgpu.ids
S=lnfc500,lnqkv500,out500,proj500
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/prof4i/$c -o run -- \
    python3 scripts/gemm_micro.py 1 $S > gpurun_out/prof4i/$c.log 2>&1 || exit $?
done
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/prof4i/MFMA -o run -- \
  python3 scripts/gemm_micro.py 1 $S > gpurun_out/prof4i/MFMA.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/prof4i $S gpurun_out/r04_i_gemm_traffic.json || exit $?
cp gpurun_out/r04_i_gemm_traffic.json profiles/
timeout -k 10 700 python bench.py --steps 20 --warmup 3 > gpurun_out/r4i_bench.log 2> gpurun_out/r4i_bench.err || exit $?
tail -1 gpurun_out/r4i_bench.log | cut -c1-1500
echo done
