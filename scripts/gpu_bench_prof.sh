set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r03p_bench.log 2>&1; rc=$?; tail -1 gpurun_out/r03p_bench.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03p_prof -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-single-window > gpurun_out/r03p_prof.log 2>&1 || exit 1
bash scripts/pmc_pass.sh r03p 48 > gpurun_out/r03p_pmc.log 2>&1; rc=$?; grep hbm_bytes gpurun_out/r03p_traffic.json; exit $rc
