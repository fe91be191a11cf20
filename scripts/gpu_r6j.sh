# r06 j: the MX c_proj (K = 4096, N = 1024: a 4-MB e4m3 panel) -- per-tile vs persistent, m-major vs
# n-tile groups; c_fc / qkv on the new default (groups of 6); MX tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6j
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx.py -q --timeout 200 --timeout-method thread \
  > gpurun_out/r6j/pytest_mx.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r6j/pytest_mx.log | tail -20; exit 1; }
tail -1 gpurun_out/r6j/pytest_mx.log
timeout -k 10 400 python3 scripts/mx_persist_micro.py 10 proj p0:2,p0:1,p2:-1,p2:2,p2:1 > gpurun_out/r6j/mx_proj.log 2>&1 || { tail -20 gpurun_out/r6j/mx_proj.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6j/mx_proj.log
timeout -k 10 300 python3 scripts/mx_persist_micro.py 10 fc8,qkv -1 > gpurun_out/r6j/mx_default.log 2>&1 || { tail -20 gpurun_out/r6j/mx_default.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6j/mx_default.log
echo done
