#!/bin/bash
# persistent halo grid at BN 128: parity against one block per patch, GPU tests, VAE conv
# A/B and same-box step / encode / decode A/B (LS_HALO_PT)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/halo_pt_check.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04m_pt_check.txt || exit 1
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread -k "not headline" > gpurun_out/r04m_gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04m_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for m in dma nopt; do
    GEMM_ONLY="vae conv" GEMM_EPI=aff timeout -k 10 300 python -u scripts/gemm_bench.py $m@48 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r04m_vae_ab.txt || exit 1
  done
done
o=gpurun_out/r04m_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py 48 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2; do
  run LS_HALO_PT=1 || exit 1
  run LS_HALO_PT=0 || exit 1
done
exit 0
