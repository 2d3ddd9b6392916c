# usage: bash scripts/gpu_quick.sh "<gemm modes>" [attn]   -- gpu tests, then microbenchmarks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/microbench.sh "$@"
