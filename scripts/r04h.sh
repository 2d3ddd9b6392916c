#!/bin/bash
# register-staged operand loads (tuning key 11) vs LDS-DMA: correctness, then graph-timed A/B at 48 windows
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r04h_ab.txt
timeout -k 10 120 python -u scripts/rs_check.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04h_check.txt || exit 1
for r in 1 2; do
  for mode in dma rs; do
    GEMM_ONLY="out0,out1,out2,qkv0,qkv2,geglu1,ff2_0,ff2_1,ff2_2,plain0" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py $mode@48 2>&1 | grep -v amdgpu.ids | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
  for mode in nohalo nohalo+rs; do
    GEMM_ONLY="conv0,conv1,conv2,conv up0" timeout -k 10 200 python -u scripts/gemm_bench.py $mode@48 2>&1 | grep -v amdgpu.ids | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
