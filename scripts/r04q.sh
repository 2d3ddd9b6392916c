#!/bin/bash
# next-K-tile DMA issued after the barrier, behind the fragment reads (ILV) vs before the
# wait (libls_hip_ab.so = c6aead6), same box: GEMM tests, short-K micro-bench, step A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread -k "not headline" > gpurun_out/r04q_gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r04q_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for m in "ilv" "ab"; do
    if [ "$m" = ab ]; then export LS_HIP_LIB=latentsync_amd/libls_hip_ab.so; else unset LS_HIP_LIB; fi
    GEMM_ONLY="out0,out1,out2,ff2_0,ff2_1,ff2_2,qkv0,qkv2,geglu1,conv up0" GEMM_EPI=res timeout -k 10 300 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/$m /" | tee -a gpurun_out/r04q_gemm_ab.txt || exit 1
  done
done
unset LS_HIP_LIB
o=gpurun_out/r04q_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py 48 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2; do
  run LS_NOTHING=1 || exit 1
  run LS_HIP_LIB=latentsync_amd/libls_hip_ab.so || exit 1
done
exit 0
