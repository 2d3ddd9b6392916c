set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03o_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r03o_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r03o_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r03o_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r03o_bench.log 2>&1; rc=$?; tail -1 gpurun_out/r03o_bench.log | cut -c1-200; exit $rc
