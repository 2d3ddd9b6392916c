# fp8 attention: parity tests, configs[4] windows (bf16 / fp8 attention) and the
# attention micro-bench at configs[4] / configs[1] shapes, bf16 vs fp8.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -v -s --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1
rc=$?; grep -E "fp8 attention|passed|failed|Error|error" gpurun_out/fp8_tests.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -k configs4 -v -s --timeout 300 --timeout-method thread > gpurun_out/fp8_c4.log 2>&1
rc=$?; grep -E "rel_err|per-pixel|passed|failed|Error" gpurun_out/fp8_c4.log | tail -20; [ $rc -ne 0 ] && exit $rc
NO_SDPA=1 CFG4=1 WINDOWS=4 timeout -k 10 120 python -u scripts/attn_bench.py > gpurun_out/fp8_bench.log 2>&1 && \
NO_SDPA=1 CFG4=1 WINDOWS=4 ATTN_FP8=1 timeout -k 10 120 python -u scripts/attn_bench.py >> gpurun_out/fp8_bench.log 2>&1 && \
NO_SDPA=1 WINDOWS=16 ATTN_ONLY=spatial timeout -k 10 120 python -u scripts/attn_bench.py >> gpurun_out/fp8_bench.log 2>&1 && \
NO_SDPA=1 WINDOWS=16 ATTN_ONLY=spatial ATTN_FP8=1 timeout -k 10 120 python -u scripts/attn_bench.py >> gpurun_out/fp8_bench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/fp8_bench.log; exit $rc
