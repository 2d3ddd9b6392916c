# pipeline / full-size / __call__ parity on the GPU, then step timing and a short bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_fullsize.py tests/test_pipeline_call.py tests/test_call_lengths.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/kv_tests.log 2>&1
rc=$?; tail -3 gpurun_out/kv_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do timeout -k 10 200 python -u scripts/step_ab.py 16 256 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-window > gpurun_out/kv_bench.log 2>&1 || exit 1
tail -1 gpurun_out/kv_bench.log | cut -c1-200
