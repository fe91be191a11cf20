# r04 ao: fused-residual GEMMs with non-temporal x16 loads / stores (probe of L2 pollution of the weight panel)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gemm_micro.py 10 resout500,resproj500 > gpurun_out/r4ao_micro.log 2>&1 || exit $?
cat gpurun_out/r4ao_micro.log
