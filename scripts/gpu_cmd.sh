set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "attention" --timeout 120 --timeout-method thread > gpurun_out/w3_tests.log 2>&1; rc=$?; tail -3 gpurun_out/w3_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q -m gpu -k "vae" --timeout 120 --timeout-method thread > gpurun_out/w3_vae.log 2>&1; rc=$?; tail -3 gpurun_out/w3_vae.log; exit $rc
