#!/bin/bash
# round 5: 4-wave row blocks, two per CU (LS_RB_NW4 bits 1: K = 320, 2: K = 640 two-fragment):
# parity with both on (ops, blocks, UNet tests), the row-block shapes A/B, whole step A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LS_RB_NW4=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py tests/test_gpu_unet.py tests/test_gpu_temporal.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05m_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05m_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r05m_rb_ab.txt
S="qkv0,geglu0,out0,plain0,geglu1"
for r in 1 2; do
  for nw in 0 3; do
    LS_RB_NW4=$nw GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/nw4=$nw /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
o=gpurun_out/r05m_step_ab.txt
for r in 1 2; do
  for nw in 0 1 3; do
    LS_RB_NW4=$nw timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/nw4=$nw /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
