#!/bin/bash
# round 5: grouped raster sweep on the 256x256 shapes beyond the K <= 1920 rule (LS_GEMM_GM
# overrides every tile; 0 = the default rule)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r05w_gm_sweep.txt
rm -f $o
for r in 1 2; do
  for gm in 0 1 2 4 8; do
    LS_GEMM_GM=$gm GEMM_ONLY="geglu2,qkv2,sc2b,sc2c,sc3,conv2,conv3,ff2_3,geglu1,qkv0" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/gm=$gm /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
