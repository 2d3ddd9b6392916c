set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "rowblock or layernorm_folded or linear" --timeout 120 --timeout-method thread > gpurun_out/p14_tests.log 2>&1
rc=$?; tail -2 gpurun_out/p14_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/debug_rb3.py > gpurun_out/p14_det.log 2>&1 || exit 1
GEMM_EPI=res GEMM_ONLY=out0 timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 dma+norb@8 > gpurun_out/p14_gemm.log 2>&1
