#!/bin/bash
# round 5: the AMDGPU machine scheduler strategy for the whole library -- default vs
# max-ilp vs max-memory-clause (libls_hip_<tag>.so, scripts/build_flags_ab.sh): whole step
# (+ encode / decode) and the main GEMM shapes, same box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r05q_step_ab.txt
rm -f $o
for r in 1 2; do
  for v in default ilp mmc itilp; do
    if [ $v = default ]; then L=latentsync_amd/libls_hip.so; else L=latentsync_amd/libls_hip_$v.so; fi
    LS_HIP_LIB=$L timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/$v-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
o=gpurun_out/r05q_gemm_ab.txt
rm -f $o
for v in default ilp mmc itilp; do
  if [ $v = default ]; then L=latentsync_amd/libls_hip.so; else L=latentsync_amd/libls_hip_$v.so; fi
  LS_HIP_LIB=$L GEMM_ONLY="conv0,conv1,conv2,qkv0,out0,out1,out2,ff2_1,geglu1,geglu2,vae conv 128 256,vae conv 512 64" GEMM_EPI=res timeout -k 10 300 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
