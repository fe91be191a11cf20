cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/rank_micro.py 3 > gpurun_out/rank_micro.log 2>&1; rc=$?
head -4 gpurun_out/rank_micro.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/mirror_micro.py > gpurun_out/mirror_micro.log 2>&1; rc=$?
tail -8 gpurun_out/mirror_micro.log; exit $rc
