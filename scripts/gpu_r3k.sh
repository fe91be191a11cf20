cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=r03_v3 bash scripts/gpu_fp8_traffic.sh || exit $?
bash scripts/gpu_configs_r2.sh
