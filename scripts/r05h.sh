#!/bin/bash
# round 5: the tree's GPU tests (non-headline) + the configs[2] 16-frame window, then a
# same-box A/B of the static half-block priority (libls_hip_ab.so: -DLS_PRIO_HALF=0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "not headline" --timeout 200 --timeout-method thread > gpurun_out/r05h_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r05h_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r05h_prio_ab.txt
S="conv0,conv1,vae conv 128 256,vae conv 256 128,out0,qkv0"
for r in 1 2; do
  GEMM_ONLY="$S" GEMM_EPI=aff,res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/prio /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 120 python -u scripts/ff_one.py 10 2>&1 | grep -v amdgpu.ids | sed "s/^/prio /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so GEMM_ONLY="$S" GEMM_EPI=aff,res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/noprio /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 120 python -u scripts/ff_one.py 10 2>&1 | grep -v amdgpu.ids | sed "s/^/noprio /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
o=gpurun_out/r05h_step_ab.txt
for r in 1 2 3; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/prio-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/noprio-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -s -q -m gpu -k "headline and 16-10" --timeout 500 --timeout-method thread > gpurun_out/r05h_headline.log 2>&1; rc=$?; grep -E "headline-depth|per-pixel|passed|failed" gpurun_out/r05h_headline.log; exit $rc
