# r05 e: where the rank fold's slab merge spends its time (probes: no slab loads / no insertions)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5e
for A in 0 1 2; do
  MICLIP_FOLD_ABL=$A timeout -k 10 120 python -u scripts/rank_stamp.py > gpurun_out/r5e/rank_stamp_abl$A.log 2>&1 || exit $?
  echo "== ABL $A"; grep -v amdgpu.ids gpurun_out/r5e/rank_stamp_abl$A.log | grep -A3 "N 1000000\|N 125000" | head -12
  grep "final ticket" gpurun_out/r5e/rank_stamp_abl$A.log
done
echo done
