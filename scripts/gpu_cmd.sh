set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "feedforward" --timeout 120 --timeout-method thread > gpurun_out/ff2_tests.log 2>&1; rc=$?; tail -1 gpurun_out/ff2_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab.sh fft2 env:LS_FUSED_FF=0 trace | head -12
