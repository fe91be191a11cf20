# r06 d: the persistent MX-fp8 ping-pong -- bit-identity tests, the configs[4] shapes micro, the fp8
# tower tests, then configs[4] (one 125k-frame L/14@336 MX-fp8 shard x 1000 queries)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6d
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py "tests/test_gpu_encode.py::test_encode_fp8_weights" \
  "tests/test_gpu_encode.py::test_last_block_on_cls_rows_bit_identical" "tests/test_gpu_encode.py::test_last_block_cls_rows_across_chunks" \
  tests/test_gpu_config_scale.py -q -rA --timeout 300 --timeout-method thread > gpurun_out/r6d/pytest_mx.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r6d/pytest_mx.log | tail -30; exit 1; }
tail -2 gpurun_out/r6d/pytest_mx.log
timeout -k 10 300 python3 scripts/mx_persist_micro.py 10 > gpurun_out/r6d/mx_persist_micro.log 2>&1 || { tail -20 gpurun_out/r6d/mx_persist_micro.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6d/mx_persist_micro.log
timeout -k 10 500 python bench.py --model ViT-L/14@336px --weights fp8 --frames 125000 --queries 1000 --steps 1 --warmup 1 \
  --no-cpu-baseline --no-rank-roofline > gpurun_out/r6d/config4.log 2> gpurun_out/r6d/config4.err || { tail -20 gpurun_out/r6d/config4.err; exit 1; }
tail -1 gpurun_out/r6d/config4.log | cut -c1-400
echo done
