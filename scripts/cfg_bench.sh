# Builder-run bench lines for BASELINE.json configs[2] (CFG, 50 steps) and configs[4] (512^2;
# bf16 attention by default, and the fp8 P.V option for the A/B), with the bounded CPU baseline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --config 2 --steps 2 > gpurun_out/cfg2_bench.log 2>&1 || exit 1
tail -1 gpurun_out/cfg2_bench.log | cut -c1-160
timeout -k 10 900 python -u bench.py --config 4 --steps 2 > gpurun_out/cfg4_bench.log 2>&1 || exit 1
tail -1 gpurun_out/cfg4_bench.log | cut -c1-160
timeout -k 10 300 python -u bench.py --config 4 --steps 2 --attn-precision fp8 --no-cpu-baseline --no-single-window > gpurun_out/cfg4_fp8_bench.log 2>&1 || exit 1
tail -1 gpurun_out/cfg4_fp8_bench.log | cut -c1-160
