#!/bin/bash
# round-5 start: short-K K = C projections on the current tree (default tiles vs forced
# 256x256 / 128x128, with the residual), then PMC of out2 (default + 256x256) and of the
# 128-channel VAE halo conv (VERDICT r04 'next' 2: a post-change PMC)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r05a_shortk.txt
for r in 1 2; do
  for mode in dma t5 t1; do
    GEMM_ONLY="out0,out1,out2,qkv2" GEMM_EPI=res timeout -k 10 150 python -u scripts/gemm_bench.py $mode@48 2>&1 | grep -v amdgpu.ids | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
SHAPE="49152 1280 1280 1 1" bash scripts/gemm_pmc.sh r05a_out2 "0 5" || exit 1
SHAPE="16777216 1152 128 3 1" AFF=1 bash scripts/gemm_pmc.sh r05a_h128 "0" || exit 1
exit 0
