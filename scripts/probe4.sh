set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/boxinfo.sh > gpurun_out/p4_box.log 2>&1
GEMM_ONLY=qkv0,out0,conv0 timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 dma+ab58@8 torch@8 >> gpurun_out/p4_box.log 2>&1
