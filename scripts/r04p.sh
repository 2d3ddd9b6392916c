#!/bin/bash
# restored (non-persistent) halo kernel + epilogue short path vs ae9a335's ls_gemm.hip
# (libls_hip_ab.so, RP on), same box: GPU tests, step / encode / decode, conv micro-bench;
# then a windows-per-batch probe (step_ab at 64 windows)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread -k "not headline" > gpurun_out/r04p_gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r04p_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r04p_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py ${NW:-48} 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2; do
  run LS_HALO_RP=1 || exit 1
  run LS_HIP_LIB=latentsync_amd/libls_hip_ab.so LS_HALO_RP=1 || exit 1
done
for m in "cur" "ab"; do
  if [ "$m" = ab ]; then export LS_HIP_LIB=latentsync_amd/libls_hip_ab.so; else unset LS_HIP_LIB; fi
  GEMM_ONLY="vae conv,conv0,conv1" GEMM_EPI=aff timeout -k 10 300 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/$m /" | tee -a gpurun_out/r04p_conv_ab.txt || exit 1
done
unset LS_HIP_LIB
NW=64 run LS_HALO_RP=1 || exit 1
exit 0
