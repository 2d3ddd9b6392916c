#!/bin/bash
# epilogue short path (bias + residual only) vs the general arithmetic (LS_GEMM_ABLATE=8),
# same box, 48 windows; then the GEMM micro-bench of the short-K shapes both ways
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread -k "not headline" > gpurun_out/r04l_gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04l_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r04l_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py 48 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2; do
  run LS_GEMM_ABLATE=0 || exit 1
  run LS_GEMM_ABLATE=8 || exit 1
done
for ab in 0 8; do
  GEMM_ONLY="out0,out1,out2,ff2_0,ff2_1,ff2_2,qkv2" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py ab$ab@48 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r04l_gemm_ab.txt || exit 1
done
exit 0
