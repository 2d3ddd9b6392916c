#!/bin/bash
# round 5: pair-split FeedForward (ff_pair_kernel; LS_FF_V1=1 = ff_fused_kernel) and the
# read-then-refill 256x256 K loop (libls_hip_ab.so = the same tree with -DLS_GEMM_RR=0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "feedforward or gemm or unet or blocks or conv or pipeline" --timeout 200 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r05f_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r05f_ff.txt
for r in 1 2; do
  timeout -k 10 120 python -u scripts/ff_one.py 10 2>&1 | grep -v amdgpu.ids | sed "s/^/pair /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_FF_V1=1 timeout -k 10 120 python -u scripts/ff_one.py 10 2>&1 | grep -v amdgpu.ids | sed "s/^/v1 /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
o=gpurun_out/r05f_rr_big.txt
S="geglu2,qkv2,ff2_2,out2,conv2,conv3,vae conv 512 64,geglu1"
for r in 1 2; do
  GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/RR /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/noRR /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
o=gpurun_out/r05f_step_ab.txt
for r in 1 2; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/A-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_FF_V1=1 timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/ffv1-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/noRR-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u scripts/serve_latency.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05f_serve_latency.txt; exit $?
