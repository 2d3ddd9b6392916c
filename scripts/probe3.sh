set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GEMM_ONLY=qkv0,out0,ff2_0,conv0,geglu0,geglu1 timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 dma+ab6@8 dma+ab14@8 dma+ab58@8 torch@8 > gpurun_out/p3_gemm.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/step_calls.py 8 > gpurun_out/p3_calls.log 2>&1
