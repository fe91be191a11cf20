# r06 u: the B/32 flash attention with its V^T fragment reads batched (A/B MICLIP_ATTN_SHORT=6)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6u; mkdir -p $D
ATTN_SHORT_MODES=vb timeout -k 10 300 python3 scripts/attn_micro.py 20 B/32c,B/32 > $D/attn_micro.log 2>&1 || { tail -20 $D/attn_micro.log; exit 1; }
grep -v amdgpu.ids $D/attn_micro.log
echo done
