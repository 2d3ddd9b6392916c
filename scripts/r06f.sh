#!/bin/bash
# round 6: ff_chain image ring (new, default lib) vs two-stage projections (libls_hip_ab.so): parity, kernel, step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "ff_chain" -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r06f_tests.log 2>&1; rc=$?; grep -E "rel|passed|failed|Error" gpurun_out/r06f_tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r06f_ab.txt
rm -f $o
for r in 1 2; do
  timeout -k 10 300 python -u scripts/ff_chain_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/new-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/ff_chain_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/old-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2 3; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/new-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/old-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
