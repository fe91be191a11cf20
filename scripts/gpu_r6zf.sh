# r06 zf: the final tree -- smoke, the fp32 tower / attention / MX / small-tile tests, the bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6zf; mkdir -p $D
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_mx.py tests/test_gpu_rk_flow.py tests/test_gpu_flows.py tests/test_gpu_encode.py -q --timeout 300 --timeout-method thread \
  > $D/pytest.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $D/pytest.log | tail -20; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $D/bench.log 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$D/bench.log').read().strip().splitlines()[-1]);p=d['parity_mode'];print('headline',d['value'],d['ms_per_step'],d['roofline']['frac'],'parity',p['value'],p['ms_per_step'])"
echo done
