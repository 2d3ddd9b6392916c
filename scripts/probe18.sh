set -o pipefail
mkdir -p gpurun_out
GEMM_EPI=res GEMM_ONLY=conv0,conv1,conv2,"conv up0" timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 > gpurun_out/p18_gemm.log 2>&1
