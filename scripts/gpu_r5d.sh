# r05 d: rank fold stamps inside the merge; c_fc packed-add GELU and full-line NT stores A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5d
timeout -k 10 120 python -u scripts/rank_stamp.py > gpurun_out/r5d/rank_stamp.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5d/rank_stamp.log
export LN_FLAGS=1
timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnfc500 44,300,174,430 > gpurun_out/r5d/lnfc.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnfc500 44,300,174,430 >> gpurun_out/r5d/lnfc.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gemm_micro.py 10 lnqkv500 0,130 > gpurun_out/r5d/lnqkv.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5d/lnfc.log gpurun_out/r5d/lnqkv.log
echo done
