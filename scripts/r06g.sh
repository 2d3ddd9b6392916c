#!/bin/bash
# round 6: VAE halo patch form A/B on the current tree (16x8 two blocks per CU, default, vs 16x16)
set -o pipefail
mkdir -p gpurun_out
o=gpurun_out/r06g_vae_ab.txt
rm -f $o
for r in 1 2 3; do
  for t in 1 0; do
    LS_DIAG_BUILD=1 LS_TUNE=16=$t timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/th8=$t-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
