#!/bin/bash
# round 6: halo conv column sums from per-thread register partials (default) vs HEAD ls_gemm.hip (ab):
# halo parity, column-sum cost per shape, step / encode / decode A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r06v_tests.log 2>&1; rc=$?; grep -E "passed|failed|Error" gpurun_out/r06v_tests.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_pipeline.py -k "not engines_dropped" -x -q --timeout 300 --timeout-method thread >> gpurun_out/r06v_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r06v_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r06v_ab.txt
rm -f $o
timeout -k 10 300 python -u scripts/cs_cost.py 2>&1 | grep -v amdgpu.ids | sed "s/^/regp /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/cs_cost.py 2>&1 | grep -v amdgpu.ids | sed "s/^/head /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/regp-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/head-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
