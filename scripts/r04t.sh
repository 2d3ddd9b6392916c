#!/bin/bash
# halo conv at N = 640: 160-channel tiles (2-slot weight ring) vs 128-channel tiles (3 slots)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for m in dma bn128; do
    GEMM_ONLY="conv1" GEMM_EPI=aff timeout -k 10 200 python -u scripts/gemm_bench.py $m@48 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r04t_bn_ab.txt || exit 1
  done
done
exit 0
