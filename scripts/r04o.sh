#!/bin/bash
# same-box: current tree (persistent halo at BN 128, epilogue short path) vs the pre-persistent
# ls_gemm.hip of ae9a335 (libls_hip_ab.so, RP on) -- step / encode / decode and VAE convs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r04o_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py 48 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2; do
  run LS_HALO_PT=1 || exit 1
  run LS_HIP_LIB=latentsync_amd/libls_hip_ab.so LS_HALO_RP=1 || exit 1
  run LS_HALO_PT=0 || exit 1
done
for m in "dma" "nopt" "ab"; do
  if [ "$m" = ab ]; then export LS_HIP_LIB=latentsync_amd/libls_hip_ab.so; mm=dma; else unset LS_HIP_LIB; mm=$m; fi
  GEMM_ONLY="vae conv,conv0,conv1" GEMM_EPI=aff timeout -k 10 300 python -u scripts/gemm_bench.py $mm@48 2>&1 | grep -v amdgpu.ids | sed "s/^/$m /" | tee -a gpurun_out/r04o_vae_ab.txt || exit 1
done
exit 0
