set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/p11_tests.log 2>&1
rc=$?; tail -3 gpurun_out/p11_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/attn_bench.py > gpurun_out/p11_attn.log 2>&1 || exit 1

