set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p22_tests.log 2>&1
rc=$?; tail -3 gpurun_out/p22_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/debug_det2.py > gpurun_out/p22_det.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/step_calls.py 8 > gpurun_out/p22_calls.log 2>&1
