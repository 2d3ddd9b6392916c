set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "rowblock or layernorm_folded or linear" --timeout 120 --timeout-method thread > gpurun_out/p19_tests.log 2>&1
rc=$?; tail -2 gpurun_out/p19_tests.log; [ $rc -ne 0 ] && exit $rc
GEMM_EPI=ln GEMM_ONLY=geglu1,ff2_1 timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 dma+norb@8 > gpurun_out/p19_gemm.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/step_calls.py 8 > gpurun_out/p19_calls.log 2>&1
