set -o pipefail
mkdir -p gpurun_out
for w in 8 16; do
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-single-window --windows-per-batch $w >> gpurun_out/p23.log 2>&1 || exit 1
done
