#!/bin/bash
# halo conv with the next tap's A fragments read before the tap barrier vs HEAD
# (libls_hip_ab.so), same box: GPU tests, conv micro-bench, step / encode / decode
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread -k "not headline" > gpurun_out/r04v_gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r04v_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for m in "cur" "ab"; do
    if [ "$m" = ab ]; then export LS_HIP_LIB=latentsync_amd/libls_hip_ab.so; else unset LS_HIP_LIB; fi
    GEMM_ONLY="conv0,conv1,vae conv 128 256,vae conv 512 64,vae conv 256 128" GEMM_EPI=aff timeout -k 10 300 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/$m /" | tee -a gpurun_out/r04v_conv_ab.txt || exit 1
  done
done
unset LS_HIP_LIB
o=gpurun_out/r04v_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py 48 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2; do
  run LS_NOTHING=1 || exit 1
  run LS_HIP_LIB=latentsync_amd/libls_hip_ab.so || exit 1
done
exit 0
