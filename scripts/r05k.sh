#!/bin/bash
# round 5: the 128-column halo conv on 16 x 8 patches, two blocks per CU (LS_HALO_TH8,
# tuning key 16): parity (both forms), the VAE conv shapes A/B, whole step + VAE A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05k_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05k_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r05k_halo_ab.txt
S="vae conv,conv0"
for r in 1 2; do
  for th in 1 0; do
    LS_HALO_TH8=$th GEMM_ONLY="$S" GEMM_EPI=aff,res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/th8=$th /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
o=gpurun_out/r05k_step_ab.txt
for r in 1 2; do
  for th in 1 0; do
    LS_HALO_TH8=$th timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/th8=$th /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
