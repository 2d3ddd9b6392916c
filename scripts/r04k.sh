#!/bin/bash
# after the halo transform / pack2 / weight-descriptor changes: GPU tests (non-headline),
# halo GN on/off/RP A/B, then the same-box step A/Bs (r04j)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread -k "not headline" > gpurun_out/r04k_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04k_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/halo_rp_check.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04k_rp_check.txt || exit 1
o=gpurun_out/r04k_gn_ab.txt
for r in 1 2; do
  for m in "aff dma" "none dma" "aff hrp"; do
    set -- $m
    GEMM_ONLY="conv0,conv1,vae conv" GEMM_EPI=$1 timeout -k 10 300 python -u scripts/gemm_bench.py $2@48 2>&1 | grep -v amdgpu.ids | sed "s/^/$1 /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
  GEMM_ONLY="vae conv 512" GEMM_EPI=aff timeout -k 10 300 python -u scripts/gemm_bench.py nohalo@48 2>&1 | grep -v amdgpu.ids | sed "s/^/aff /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
bash scripts/r04j.sh
