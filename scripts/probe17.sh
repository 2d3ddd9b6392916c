set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv or gemm or linear" --timeout 120 --timeout-method thread > gpurun_out/p17_tests.log 2>&1
rc=$?; tail -2 gpurun_out/p17_tests.log; [ $rc -ne 0 ] && exit $rc
GEMM_ONLY=conv timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 > gpurun_out/p17_gemm.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/step_calls.py 8 > gpurun_out/p17_calls.log 2>&1
