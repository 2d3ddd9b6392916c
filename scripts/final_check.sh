set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-final}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "not headline" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
# the headline-depth windows (configs[1] 16x20, CFG 4x20, configs[2] depth 4x50) with their figures printed
[ -z "$SKIP_HEADLINE" ] && timeout -k 10 1000 python -u -m pytest tests/test_gpu_fullsize.py -x -s -q -m gpu -k headline --timeout 900 --timeout-method thread > gpurun_out/${TAG}_headline.log 2>&1; rc=$?; [ -z "$SKIP_HEADLINE" ] && { grep -E "headline-depth|per-pixel|passed|failed" gpurun_out/${TAG}_headline.log; [ $rc -ne 0 ] && exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_bench.log | cut -c1-200; exit $rc
