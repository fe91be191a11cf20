# gemm_8q tile order: default raster vs n-tiles walked in groups (variants 12x), timing + clock/MFMA busy + FETCH
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/grp
timeout -k 10 400 python -u scripts/gemm_micro.py 10 fc500,qkv500,out500,proj500 0,132,133,134,136 > gpurun_out/grp/micro.log 2>&1 || exit $?
cat gpurun_out/grp/micro.log
for V in 0 134 136; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES FETCH_SIZE --output-format csv -d gpurun_out/grp/v$V -o run -- \
    python3 scripts/gemm_micro.py 1 fc500,qkv500 $V > gpurun_out/grp/v$V.log 2>&1 || exit $?
done
