#!/bin/bash
# round 5: grouped tile raster (LS_GEMM_GM = row-blocks per group) on the short-K shapes that
# re-read their A band once per N tile (out1 / ff2_1 on 128x160: 4 N tiles; out2 / sc2b on
# 256x256: 5), same box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r05s_gm_ab.txt
rm -f $o
for r in 1 2; do
  for gm in 0 2 4 8 16; do
    LS_GEMM_GM=$gm GEMM_ONLY="out1,ff2_1,out2,sc2b,ff2_2" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/gm=$gm /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
