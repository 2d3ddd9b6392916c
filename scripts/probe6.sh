set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GEMM_EPI=ln GEMM_ONLY=geglu,qkv timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 dma+t9@8 dma+t1@8 dma+t5@8 > gpurun_out/p6_gemm.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/attn_bench.py > gpurun_out/p6_attn.log 2>&1
