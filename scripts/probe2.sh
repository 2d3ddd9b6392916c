set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GEMM_ONLY=qkv0,out0,ff2_0,conv0 timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 dma+ab2@8 dma+ab6@8 dma+ab14@8 dma+ab10@8 dma+ab48@8 dma+ab56@8 dma+ab58@8 dma+ab62@8 dma+ab24@8 > gpurun_out/p2_gemm.log 2>&1 || exit 1
GEMM_ONLY=qkv0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d gpurun_out/p2_pmc -o run -- python3 scripts/gemm_bench.py dma@8 dma+ab6@8 > gpurun_out/p2_pmc.log 2>&1
