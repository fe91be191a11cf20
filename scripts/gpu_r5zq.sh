# r05 zq: locate the fp32 tower's non-finite rows: 8-phase GEMMs with neither / either of the CLS-row block and the dedup
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5zq
export F32_NO_EXIT=1
F32_VARIANTS=ppnocls,m4,A,d8,C,B,8q timeout -k 10 200 python3 scripts/f32_micro.py 300 1 > gpurun_out/r5zq/f32_m.log 2>&1 || { tail -30 gpurun_out/r5zq/f32_m.log; exit 1; }
grep -v "amdgpu.ids\|RuntimeWarning\|api.load" gpurun_out/r5zq/f32_m.log
echo done
