# r04 at: configs[3] (one 125k-frame B/32 shard x 32 queries) on the final tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cfg4
timeout -k 10 300 python bench.py --model ViT-B/32 --frames 125000 --queries 32 --steps 2 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/cfg4/c3at.log 2>&1 || exit $?
tail -1 gpurun_out/cfg4/c3at.log > gpurun_out/cfg4/c3at.json
python3 -c "import json; d=json.load(open('gpurun_out/cfg4/c3at.json')); print('c3', d['value'], d['ms_per_step'])"
