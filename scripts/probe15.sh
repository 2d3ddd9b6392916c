set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/p15_counters.txt 2>&1 || true
ATTN_ONLY="spatial L0" NO_SDPA=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/p15_a -o run -- python3 scripts/attn_bench.py > gpurun_out/p15_a.log 2>&1 || exit 1
ATTN_ONLY="spatial L0" NO_SDPA=1 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/p15_b -o run -- python3 scripts/attn_bench.py > gpurun_out/p15_b.log 2>&1
