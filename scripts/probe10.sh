set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/p10_tests.log 2>&1
rc=$?; tail -3 gpurun_out/p10_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/debug_det2.py > gpurun_out/p10_det.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/step_calls.py 8 > gpurun_out/p10_calls.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-single-window > gpurun_out/p10_bench.log 2>&1
