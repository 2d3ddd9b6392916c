#!/bin/bash
# round 6: K = 640 residual linears on the row-block GEMM (tuning key 20) vs the tiled 128 x 160 kernel
set -o pipefail
mkdir -p gpurun_out
o=gpurun_out/r06p_ab.txt
rm -f $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "rowblock or linear" -x -q --timeout 200 --timeout-method thread > gpurun_out/r06p_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r06p_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  LS_DIAG_BUILD=1 LS_TUNE=20=1 timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/rb-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/tiled-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
