set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p24_tests.log 2>&1
rc=$?; tail -2 gpurun_out/p24_tests.log; [ $rc -ne 0 ] && exit $rc
GEMM_EPI=res timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 > gpurun_out/p24_gemm.log 2>&1
