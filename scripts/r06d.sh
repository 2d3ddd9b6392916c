#!/bin/bash
# round 6: full GPU suite (not headline) + smoke + bench line with the chain in the step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "not headline" --timeout 300 --timeout-method thread > gpurun_out/r06d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06d_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r06d_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r06d_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r06d_bench.log 2>&1; rc=$?; tail -1 gpurun_out/r06d_bench.log | cut -c1-400; exit $rc
