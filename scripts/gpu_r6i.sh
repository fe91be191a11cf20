# r06 i: the persistent MX kernel's tile-order group width (the m-major walk re-fetches c_fc's 4-MB
# e4m3 weight panel: FETCH 9x the operand bytes, profiles/r06_h_fp8_gemm_traffic.json)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6i
timeout -k 10 400 python3 scripts/mx_persist_micro.py 10 fc8,qkv,out -1,2,4,8,6 > gpurun_out/r6i/mx_ng.log 2>&1 || { tail -20 gpurun_out/r6i/mx_ng.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6i/mx_ng.log
echo done
