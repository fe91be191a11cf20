# r06 c: tile-order group width re-swept on the product LN-folded in_proj / c_fc (whole-line NT
# stores since r05 changed the L2 picture): interleaved rounds in one process, maxdiff vs default
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6c
LN_FLAGS=1 timeout -k 10 300 python3 scripts/gemm_micro.py 20 lnqkv500 0,20003,20005,20004,20001 > gpurun_out/r6c/ng_qkv.log 2>&1 || { tail -20 gpurun_out/r6c/ng_qkv.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6c/ng_qkv.log
LN_FLAGS=1 timeout -k 10 300 python3 scripts/gemm_micro.py 20 lnfc500 0,19999,20004,20003,20002 > gpurun_out/r6c/ng_fc.log 2>&1 || { tail -20 gpurun_out/r6c/ng_fc.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6c/ng_fc.log
echo done
