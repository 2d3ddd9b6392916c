set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p16_tests.log 2>&1
rc=$?; tail -2 gpurun_out/p16_tests.log; [ $rc -ne 0 ] && exit $rc
NO_SDPA=1 timeout -k 10 200 python -u scripts/attn_bench.py > gpurun_out/p16_attn.log 2>&1
