# Secondary BASELINE configs on one GPU (parity-test cases, not the bench line):
# configs[2] ViT-L/14 bf16 (x256 queries) and configs[4]'s model ViT-L/14@336px (x1000 queries).
mkdir -p gpurun_out/cfg
timeout -k 10 400 python bench.py --model ViT-L/14 --frames ${L14_FRAMES:-20000} --queries 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cfg/l14.log 2>&1 || exit $?
tail -1 gpurun_out/cfg/l14.log
timeout -k 10 400 python bench.py --model ViT-L/14@336px --frames ${L336_FRAMES:-5000} --queries 1000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cfg/l336.log 2>&1 || exit $?
tail -1 gpurun_out/cfg/l336.log
