# r05 za: L/14 c_fc default tile order (one group per XCD) against m-major and forced groups of 2, same box
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5za
export LN_FLAGS=1
for ng in def -1 2 def -1; do
  if [ "$ng" = def ]; then unset MICLIP_8Q_NG; else export MICLIP_8Q_NG=$ng; fi
  timeout -k 10 200 python -u scripts/gemm_micro.py 5 lnfcL 942 > gpurun_out/r5za/L$ng.log 2>&1 || { cat gpurun_out/r5za/L$ng.log; exit 1; }
  echo "ng=$ng"; grep -v amdgpu.ids gpurun_out/r5za/L$ng.log
done
echo done
