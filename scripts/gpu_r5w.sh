# r05 w: L/14 attention, Q fragments loaded one tile ahead (A/B var 14)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5w
ATTN_VARS=1,14,1,14 timeout -k 10 300 python -u scripts/attn_micro.py 10 L/14c,L/14 > gpurun_out/r5w/attn.log 2>&1 || { cat gpurun_out/r5w/attn.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5w/attn.log
echo done
