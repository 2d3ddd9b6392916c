#!/bin/bash
# round 5: row-block GEMM with the residual fragments read before the chunk's MFMAs, the
# unconditional output scale and the W fragments one k-step ahead (LS_RB_PRE, default) vs
# the previous form (libls_hip_ab.so, -DLS_RB_PRE=0): parity, row-block shapes, whole step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05n_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05n_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r05n_rb_ab.txt
S="qkv0,geglu0,out0,plain0,geglu1"
for r in 1 2; do
  GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/pre /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/old /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
o=gpurun_out/r05n_step_ab.txt
for r in 1 2 3; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/pre-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/old-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
