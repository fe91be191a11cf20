# rank (tests + micro + trace) then attention (r32 tests + micro) in one call
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_rank_cert.sh || exit $?
bash scripts/gpu_attn_r32.sh || exit $?
