#!/bin/bash
# round 5: timing ablations of the row-block / tiled kernels on the short-K projections
# (diagnostics build as libls_hip_ab.so: ablation bits 2 no chunk / operand DMA, 4 no
# stores, 64 no A-row loads in the row-block kernel)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r05l_ablate.txt
rm -f $o
for ab in 0 2 4 6 64 66 68 70; do
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so GEMM_ONLY="out0,qkv0,out1,out2" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma+ab$ab@48 2>&1 | grep -v amdgpu.ids | grep -v TOTAL | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
