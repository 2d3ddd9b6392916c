set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p13_tests.log 2>&1
rc=$?; tail -2 gpurun_out/p13_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 100 python -u scripts/gn_bench.py > gpurun_out/p13.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/step_calls.py 8 > gpurun_out/p13_calls.log 2>&1
