#!/bin/bash
# round 5: (1) read-then-refill DMA GEMM K loop (A) vs the previous loop (B: libls_hip_ab.so
# built with -DLS_GEMM_RR=0); (2) 4-stage row-block ring (LS_RB_NS3=1 = 3 stages);
# (3) FeedForward ablations (LS_FF_ABLATE: 1 no W DMA, 2 no GELU, 4 no GEMM2); (4) step A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "rowblock or gemm or feedforward or gn_colsum or linear or unet or conv" --timeout 200 --timeout-method thread > gpurun_out/r05e_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r05e_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r05e_rr_ab.txt
S="out1,out2,qkv2,ff2_1,ff2_2,qkv0,sc2b"
for r in 1 2; do
  GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/RR /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/noRR /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
o=gpurun_out/r05e_rb_ab.txt
S="out0,qkv0,plain0"
for r in 1 2; do
  GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/NS4 /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_RB_NS3=1 GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/NS3 /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
o=gpurun_out/r05e_ff.txt
for ab in 0 1 2 4 3 0; do
  LS_FF_ABLATE=$ab timeout -k 10 120 python -u scripts/ff_one.py 10 2>&1 | grep -v amdgpu.ids | sed "s/^/ablate=$ab /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
o=gpurun_out/r05e_step_ab.txt
for r in 1 2; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/A-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/noRR-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_RB_NS3=1 timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/NS3-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
