# r06 v: encode_text (32 queries) with 64 x 64 tiles for the text tower's small GEMMs (A/B MICLIP_SMALL64)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6v; mkdir -p $D
timeout -k 10 300 python3 scripts/text_micro.py 32 5 > $D/text_micro.log 2>&1 || { tail -20 $D/text_micro.log; exit 1; }
grep -v -E "amdgpu.ids|RuntimeWarning|models\[k\]" $D/text_micro.log
echo done
