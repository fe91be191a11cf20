cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/v6
timeout -k 10 120 python3 scripts/gemm_micro.py 20 qkv,out,fc,proj,long 3,6 > gpurun_out/v6/micro.log 2>&1 || exit $?
cat gpurun_out/v6/micro.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/v6/FETCH_SIZE -o run -- python3 scripts/gemm_micro.py 1 fc,qkv 6 > gpurun_out/v6/f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/v6/WRITE_SIZE -o run -- python3 scripts/gemm_micro.py 1 fc,qkv 6 > gpurun_out/v6/w.log 2>&1 || exit $?
