# r04 v: secondary configs with the round-4 kernels (LN-folded bf16 towers for B/32 and L/14)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# Secondary BASELINE configs at their stated corpus sizes (one GPU = one shard for the
# 8-GPU configs): configs[2] ViT-L/14 bf16 100k frames x 256 queries; configs[3] one
# 125k-frame shard of the 1M B/32 corpus x 32 queries; configs[4] one 125k-frame shard
# of the 1M L/14@336px corpus, MX-fp8 weights, x 1000 queries.  One timed step each.
mkdir -p gpurun_out/cfg4
timeout -k 10 300 python bench.py --model ViT-B/32 --frames 125000 --queries 32 --steps 2 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/cfg4/c3.log 2>&1 || exit $?
tail -1 gpurun_out/cfg4/c3.log > gpurun_out/cfg4/c3.json
timeout -k 10 400 python bench.py --model ViT-L/14 --frames 100000 --queries 256 --steps 1 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/cfg4/c2.log 2>&1 || exit $?
tail -1 gpurun_out/cfg4/c2.log > gpurun_out/cfg4/c2.json
timeout -k 10 500 python bench.py --model ViT-L/14@336px --weights fp8 --frames 125000 --queries 1000 --steps 1 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/cfg4/c4.log 2>&1 || exit $?
tail -1 gpurun_out/cfg4/c4.log > gpurun_out/cfg4/c4.json
for c in c3 c2 c4; do python3 -c "import json; d=json.load(open('gpurun_out/cfg4/$c.json')); print('$c', d['value'], d['ms_per_step'], d['config']['workload'], d.get('mfma_frac_end_to_end'), d['roofline']['frac'] if d.get('roofline') else None)"; done
