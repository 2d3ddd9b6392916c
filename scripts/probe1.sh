set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/step_calls.py 8 > gpurun_out/p1_calls.log 2>&1 || exit 1
GEMM_ONLY=qkv0,geglu0,ff2_0,out0,conv0,geglu1,vae timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 torch@8 dma+ab2@8 dma+ab4@8 dma+ab6@8 > gpurun_out/p1_gemm.log 2>&1
