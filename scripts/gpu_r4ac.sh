# r04 ac: fused-residual GEMM timing probes (no statistics / no x16 loads) beside the product kernel
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gemm_micro.py 10 resout500,resproj500 > gpurun_out/r4ac_micro.log 2>&1 || exit $?
cat gpurun_out/r4ac_micro.log
