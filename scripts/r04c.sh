#!/bin/bash
# short-K residual projections (K = C: the out-projections at 16x16 / 8x8, 48 windows):
# where does the time go?  default vs no operand DMA / no stores / forced tiles / BK 32 /
# grouped raster / hipBLASLt, same box, graph-timed (scripts/gemm_bench.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r04c_shortk.txt
for r in ${ROUNDS:-1 2}; do
for mode in dma nodma ab4 torch t1 t2 t3 bk32 norb; do
  GEMM_ONLY="out0,out1,out2,qkv0,qkv2" GEMM_EPI=res timeout -k 10 120 python -u scripts/gemm_bench.py $mode@48 2>&1 | grep -v amdgpu.ids | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
for gm in 2 4 8; do
  LS_GEMM_GM=$gm GEMM_ONLY="out0,out1,out2,qkv0,qkv2" GEMM_EPI=res timeout -k 10 120 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/gm$gm /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
done
exit 0
