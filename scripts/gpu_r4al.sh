# r04 al: ViT-L/14 (W = 1024) with the fold + fused residual against the unfolded tower (A/B build):
# 10k frames x 256 queries, the configs[2] model at a shorter workload
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export MICLIP_LIB=ab
for v in "0 1" "1 1" "1 0"; do
  set -- $v
  MICLIP_LNFOLD=$1 MICLIP_RESFUSE=$2 timeout -k 10 400 python bench.py --model ViT-L/14 --frames 10000 --queries 256 \
    --steps 3 --warmup 1 --no-parity-mode --no-cpu-baseline --no-rank-roofline --no-kernel-timing \
    > gpurun_out/r4al_fold$1_fuse$2.log 2> gpurun_out/r4al_fold$1_fuse$2.err || exit $?
  echo "fold=$1 fuse=$2: $(tail -1 gpurun_out/r4al_fold$1_fuse$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
