#!/bin/bash
# round 6: ff_chain 32 rows per wave (one wave per SIMD) parity + kernel time + step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "ff_chain" -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r06c_tests.log 2>&1; rc=$?; grep -E "rel|passed|failed|Error" gpurun_out/r06c_tests.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ff_chain_bench.py > gpurun_out/r06c_kernel.txt 2>&1; rc=$?; cat gpurun_out/r06c_kernel.txt | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r06c_step_ab.txt
rm -f $o
for r in 1 2 3; do
  for c in 2 1; do
    LS_DIAG_BUILD=1 LS_TUNE=17=$c timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/fmr=$c-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
