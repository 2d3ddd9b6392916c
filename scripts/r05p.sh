#!/bin/bash
# round 5: FeedForward software-pipelined one GEMM1 ahead (LS_FF_PIPE=1, ff_pipe_kernel) vs
# ff_fused_kernel: parity, per-call time, whole step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LS_FF_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "feedforward" -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05p_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05p_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r05p_ff.txt
rm -f $o
for r in 1 2 3; do
  for p in 1 0; do
    LS_FF_PIPE=$p timeout -k 10 120 python -u scripts/ff_one.py 20 2>&1 | grep -v amdgpu.ids | sed "s/^/pipe=$p /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
o=gpurun_out/r05p_step_ab.txt
rm -f $o
for r in 1 2; do
  for p in 1 0; do
    LS_FF_PIPE=$p timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/pipe=$p-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
