# r05 zd: the certified rank route below its 262144-row threshold now that the merge is a ~6-us launch
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zd
export RANK_MICRO_VARIANTS=default,cert_any,default,cert_any
timeout -k 10 300 python -u scripts/rank_micro.py 5 > gpurun_out/r5zd/rank_micro.log 2>&1 || { cat gpurun_out/r5zd/rank_micro.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5zd/rank_micro.log | head -7 | cut -c1-300
echo done
