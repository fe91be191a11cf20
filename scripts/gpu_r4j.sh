# r04 j: is the LN-folded GEMM's extra time code or power?  The same kernels on operands
# with bf16-width significands (_t) against full fp16 ones; plain bf16 kernels beside them
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python scripts/gemm_micro.py 20 lnfc500,lnfc500_t,fc500,lnqkv500,lnqkv500_t,qkv500,lnfc500,fc500 > gpurun_out/r4j_gemm_micro.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4j_gemm_micro.log
