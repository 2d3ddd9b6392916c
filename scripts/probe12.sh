set -o pipefail
mkdir -p gpurun_out
for r in 8 16 32 64 128; do LS_GN_RPT=$r timeout -k 10 100 python -u scripts/gn_bench.py >> gpurun_out/p12.log 2>&1 || exit 1; done
