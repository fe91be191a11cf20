set -e
cd /root/repo
mkdir -p gpurun_out/pmc_attn
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_attn/p1 -o p1 --output-format csv -- python3 scripts/attn_micro.py 3 L/14@336,L/14 > gpurun_out/pmc_attn/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM -d gpurun_out/pmc_attn/p2 -o p2 --output-format csv -- python3 scripts/attn_micro.py 3 L/14@336,L/14 > gpurun_out/pmc_attn/p2.log 2>&1
