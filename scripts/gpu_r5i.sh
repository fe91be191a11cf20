# r05 i: the parity mode's fused c_fc split against the separate split pass (A/B build, same box),
# and the kernel trace of the product parity mode (bench --weights fp32)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5i
for F in 0 1 0 1; do
  MICLIP_LIB=ab MICLIP_F32_FUSED_SPLIT=$F timeout -k 10 300 python bench.py --weights fp32 --steps 3 --warmup 1 --no-cpu-baseline \
    --no-rank-roofline --no-kernel-timing > gpurun_out/r5i/fp32_fused$F.log 2> gpurun_out/r5i/fp32_fused$F.err || { tail -5 gpurun_out/r5i/fp32_fused$F.err; exit 1; }
  echo "fused=$F $(tail -1 gpurun_out/r5i/fp32_fused$F.log | cut -c1-120)"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5i/prof_fp32 -o bench -- \
  python3 bench.py --weights fp32 --steps 2 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-kernel-timing \
  > gpurun_out/r5i/prof_fp32.log 2>&1 || exit $?
echo done
