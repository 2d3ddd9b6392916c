# A/B of the fp8 attention variants (LS_ATTN8_VARIANT) at the configs[4] 64^2-level shape + a
# rocprofv3 kernel trace of the default variant (quantise vs attend time).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp NO_SDPA=1 CFG4=1 WINDOWS=4 ATTN_ONLY=L0
timeout -k 10 100 python -u scripts/attn_bench.py > gpurun_out/fp8ab.log 2>&1 || exit 1
for v in 0 1 2 3; do
  LS_ATTN8_VARIANT=$v ATTN_FP8=1 timeout -k 10 100 python -u scripts/attn_bench.py 2>&1 | sed "s/^/variant $v: /" >> gpurun_out/fp8ab.log || exit 1
done
grep -v amdgpu.ids gpurun_out/fp8ab.log
ATTN_FP8=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/fp8prof -o run -- python3 -u scripts/attn_bench.py > gpurun_out/fp8prof.log 2>&1 || exit 1
python3 scripts/kernel_stats.py gpurun_out/fp8prof/run_results.db | head -6
