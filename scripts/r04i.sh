#!/bin/bash
# PMC passes of the halo-tile 3x3 conv: VAE 128 ch at 256^2 and the UNet's 320 ch at 32^2
# (GroupNorm affine variant), plus the 128x160 1x1 residual GEMM at K = 640 for reference
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r04i_gn_ab.txt
# parity of the RP halo enumeration against the default one (bit-identical expected)
timeout -k 10 120 python -u scripts/halo_rp_check.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04i_rp_check.txt || exit 1
# the halo conv with and without the GroupNorm affine + SiLU on its input (GN template flag)
for r in 1 2; do
  for epi in aff none; do
    GEMM_ONLY="conv0,conv1,vae conv 128 256,vae conv 256 128" GEMM_EPI=$epi timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/$epi /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
  # halo pieces over the read pixels only (tuning key 12)
  GEMM_ONLY="conv0,conv1,vae conv 128 256,vae conv 256 128" GEMM_EPI=aff timeout -k 10 200 python -u scripts/gemm_bench.py hrp@48 2>&1 | grep -v amdgpu.ids | sed "s/^/aff /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
SHAPE="16777216 1152 128 3 1" AFF=1 bash scripts/gemm_pmc.sh r04i_h128 "0" || exit 1
SHAPE="262144 2880 320 3 1" AFF=1 bash scripts/gemm_pmc.sh r04i_h320 "0" || exit 1
exit 0
