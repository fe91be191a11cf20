# r04 av: c_fc QuickGELU stage order over the 16-row block's 16 values (flags 44) against the
# product's 8-value order (12) and none (1), interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LN_FLAGS=1 timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnfc500 12,44,1 > gpurun_out/r4av_lnfc.log 2>&1 || exit $?
LN_FLAGS=1 timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnfc500 12,44,1 >> gpurun_out/r4av_lnfc.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4av_lnfc.log
