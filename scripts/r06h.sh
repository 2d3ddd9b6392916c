#!/bin/bash
# round 6: upsample convs on the halo kernel -- parity, then step / encode / decode A/B (key 18)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_halo.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r06h_tests.log 2>&1; rc=$?; grep -E "upsample|passed|failed|Error" gpurun_out/r06h_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r06h_ab.txt
rm -f $o
for r in 1 2 3; do
  for t in 1 0; do
    LS_DIAG_BUILD=1 LS_TUNE=18=$t timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/ups=$t-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 300 python -u scripts/step_calls.py 48 256 decode > gpurun_out/r06h_decode_calls.txt 2>&1; grep "up=1" gpurun_out/r06h_decode_calls.txt | head
timeout -k 10 300 python -u scripts/step_calls.py 48 256 step > gpurun_out/r06h_step_calls.txt 2>&1; grep "up=1" gpurun_out/r06h_step_calls.txt | head
exit 0
