#!/bin/bash
# round 5: grouped raster (4 row bands) for 256x256 1x1 tiles with K <= 1920 (default) vs the
# column-fastest order (LS_GEMM_GM_SHORTK=0): shapes, whole step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r05u_gm_ab.txt
rm -f $o
for r in 1 2; do
  for g in 1 0; do
    LS_GEMM_GM_SHORTK=$g GEMM_ONLY="out2,sc2a,sc2b,qkv2,geglu2,out3,ff2_2" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/gm4=$g /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
o=gpurun_out/r05u_step_ab.txt
rm -f $o
for r in 1 2 3; do
  for g in 1 0; do
    LS_GEMM_GM_SHORTK=$g timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/gm4=$g-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
