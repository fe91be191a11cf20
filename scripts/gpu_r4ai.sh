# r04 ai: B/32 attention variants timed in interleaved rounds
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/attn_micro.py 10 B/32c,text > gpurun_out/r4ai_attn.log 2>&1 || exit $?
cat gpurun_out/r4ai_attn.log
