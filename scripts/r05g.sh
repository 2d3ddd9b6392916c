#!/bin/bash
# round 5: pair-split FeedForward (ff_pair_kernel) vs ff_fused_kernel (LS_FF_V1=1), same box;
# the time embedding computed once per batch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "feedforward or unet or blocks or pipeline or gemm" --timeout 200 --timeout-method thread > gpurun_out/r05g_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r05g_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r05g_ff.txt
for r in 1 2 3; do
  timeout -k 10 120 python -u scripts/ff_one.py 10 2>&1 | grep -v amdgpu.ids | sed "s/^/pair /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_FF_V1=1 timeout -k 10 120 python -u scripts/ff_one.py 10 2>&1 | grep -v amdgpu.ids | sed "s/^/v1 /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
o=gpurun_out/r05g_step_ab.txt
for r in 1 2 3; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/pair-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_FF_V1=1 timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/v1-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
