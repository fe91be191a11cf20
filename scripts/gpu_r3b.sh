# Round 3: the whole GPU suite + smoke, a rank_reg 8- vs 9-slot micro A/B, then the round
# measurement (PMC passes, bench, rocprof trace) of scripts/gpu_round.sh.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python scripts/rank_nb_ab.py > gpurun_out/rank_nb.log 2>&1 || exit $?
cat gpurun_out/rank_nb.log
TAG=${TAG:-r03_v1} bash scripts/gpu_round.sh
