# r04 as: the default bench line once more on another box, with the kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4as
timeout -k 10 700 python bench.py --steps 20 --warmup 3 > gpurun_out/r4as_bench.log 2> gpurun_out/r4as_bench.err || exit $?
tail -1 gpurun_out/r4as_bench.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4as -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rank-roofline --no-parity-mode > gpurun_out/prof4as/stdout.log 2>&1 || exit $?
echo done
