# r06 h: the persistent MX kernel's QuickGELU in stage order (bit-identity against the per-tile
# kernel, timing), and the PMC traffic / MFMA busy of the tower's MX-fp8 c_fc (GELU -> MX-fp8)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6h
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx.py -q -k "persistent or default_fp8" --timeout 200 --timeout-method thread \
  > gpurun_out/r6h/pytest_mx.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r6h/pytest_mx.log | tail -20; exit 1; }
tail -1 gpurun_out/r6h/pytest_mx.log
timeout -k 10 300 python3 scripts/mx_persist_micro.py 10 fc8,fc8_100k,qkv > gpurun_out/r6h/mx_persist_micro.log 2>&1 || { tail -20 gpurun_out/r6h/mx_persist_micro.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6h/mx_persist_micro.log
TAG=r06_h bash scripts/gpu_fp8_traffic.sh > gpurun_out/r6h/fp8_traffic.log 2>&1 || { tail -20 gpurun_out/r6h/fp8_traffic.log; exit 1; }
tail -2 gpurun_out/r6h/fp8_traffic.log
echo done
