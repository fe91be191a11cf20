# r04 aj: persistent short attention with the next item prefetched (A/B) -- attention tests through the
# A/B library with the variant forced, then the interleaved micro
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/attn_micro.py 10 B/32c > gpurun_out/r4aj_attn.log 2>&1 || exit $?
cat gpurun_out/r4aj_attn.log
