# r04 am: fold + fused residual for W <= 1024: encode tests, configs[2] (L/14, now folded)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cfg4
timeout -k 10 900 python -u -m pytest tests/test_gpu_encode.py -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/r4am_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4am_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --model ViT-L/14 --frames 100000 --queries 256 --steps 1 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/cfg4/c2am.log 2>&1 || exit $?
tail -1 gpurun_out/cfg4/c2am.log > gpurun_out/cfg4/c2am.json
python3 -c "import json; d=json.load(open('gpurun_out/cfg4/c2am.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['kernel'][:40], d['roofline']['frac'])"
