#!/bin/bash
# round 6 final tree (after the column-sum change), part A: every -m gpu test, the headline-depth windows, smoke
set -o pipefail
mkdir -p gpurun_out
T=r06x
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "not headline" -s --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fullsize.py -x -s -q -m gpu -k headline --timeout 900 --timeout-method thread > gpurun_out/${T}_headline.log 2>&1; rc=$?; grep -E "headline-depth|per-pixel|passed|failed" gpurun_out/${T}_headline.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${T}_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_smoke.log; exit $rc
