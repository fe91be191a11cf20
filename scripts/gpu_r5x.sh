# r05 x: tile-order group width of the LN-folded GEMMs at the ViT-L/14 shapes (K = 1024: the
# default rule finds no group whose weight panel fits 2.4 MB, so c_fc / in_proj run m-major)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5x
export LN_FLAGS=1
for ng in -1 4 2 8 -1; do
  MICLIP_8Q_NG=$ng timeout -k 10 200 python -u scripts/gemm_micro.py 5 lnfcL,lnqkvL 942 > gpurun_out/r5x/ng$ng.log 2>&1 || { cat gpurun_out/r5x/ng$ng.log; exit 1; }
  echo "ng=$ng"; grep -v amdgpu.ids gpurun_out/r5x/ng$ng.log
done
echo done
