#!/bin/bash
# A/B on one box (graph-timed, 48 windows): (1) the 256x128 3-stage tile for the short-K
# linears vs the default tiles; (2) the halo-tile 3x3 conv (GN affine + SiLU fused) vs the
# tiled conv behind a materialised ls_groupnorm_apply
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r04e_ab.txt
for r in 1 2; do
  for mode in dma t256; do
    GEMM_ONLY="out1,out2,qkv2,geglu1,ff2_1,ff2_2" GEMM_EPI=res timeout -k 10 150 python -u scripts/gemm_bench.py $mode@48 2>&1 | grep -v amdgpu.ids | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
  for mode in dma nohalo; do
    GEMM_ONLY="conv0,conv1,vae conv" GEMM_EPI=aff timeout -k 10 200 python -u scripts/gemm_bench.py $mode@48 2>&1 | grep -v amdgpu.ids | sed "s/^/aff /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
