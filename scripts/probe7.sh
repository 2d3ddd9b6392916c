set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GEMM_EPI=ln GEMM_ONLY=geglu0,plain0 timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 > gpurun_out/p7.log 2>&1 || exit 1
for w in 8 12 16; do
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-single-window --windows-per-batch $w >> gpurun_out/p7.log 2>&1 || exit 1
done
