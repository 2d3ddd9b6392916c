#!/bin/bash
# round 5: row-block epilogue interleaved with the next chunk's MFMAs by sched_group_barrier
# (LS_RB_PRE bit 8, with the branch-free scale bit 2; 11 also preloads the residual) against
# the previous form (libls_hip_ab.so, LS_RB_PRE=0): parity of the 10 build, shapes, step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LS_HIP_LIB=latentsync_amd/libls_hip_ab10.so timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05o_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05o_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r05o_rb_ab.txt
rm -f $o
S="qkv0,out0,plain0,geglu0,geglu1"
for r in 1 2; do
  for v in ab ab10 ab11; do
    LS_HIP_LIB=latentsync_amd/libls_hip_$v.so GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
o=gpurun_out/r05o_step_ab.txt
rm -f $o
for r in 1 2; do
  for v in ab ab10 ab11; do
    LS_HIP_LIB=latentsync_amd/libls_hip_$v.so timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/$v-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
