# r05 y: tile-order group width of the B/32 c_fc (default 6) and of the L/14 c_fc (default raster) re-measured
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5y
export LN_FLAGS=1
for ng in 6 2 3 4 -1 6 2; do
  MICLIP_8Q_NG=$ng timeout -k 10 200 python -u scripts/gemm_micro.py 5 lnfc500 942 > gpurun_out/r5y/ng$ng.log 2>&1 || { cat gpurun_out/r5y/ng$ng.log; exit 1; }
  echo "ng=$ng"; grep -v amdgpu.ids gpurun_out/r5y/ng$ng.log
done
for ng in 2 1 -1 2; do
  MICLIP_8Q_NG=$ng timeout -k 10 200 python -u scripts/gemm_micro.py 5 lnfcL 942 > gpurun_out/r5y/L$ng.log 2>&1 || { cat gpurun_out/r5y/L$ng.log; exit 1; }
  echo "L ng=$ng"; grep -v amdgpu.ids gpurun_out/r5y/L$ng.log
done
echo done
