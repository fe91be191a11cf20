# rocprofv3 kernel trace + stats of the bench (no PMC here; counters go in their own pass)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_stdout.log 2>&1
rc=$?
ls -R gpurun_out/prof | head -30
exit $rc
