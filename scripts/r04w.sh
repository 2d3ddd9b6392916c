#!/bin/bash
# 1x1 GEMM with the A operand straight into registers (LS_GEMM_AREG) vs the LDS-DMA kernel:
# bit-exactness, the GEMM / block / UNet GPU tests under the switch, micro-bench, step A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/areg_check.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04w_areg_check.txt || exit 1
LS_GEMM_AREG=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py tests/test_gpu_unet.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04w_gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r04w_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for m in dma areg; do
    GEMM_ONLY="out0,out1,out2,ff2_0,ff2_1,ff2_2,qkv0,qkv2,geglu1,plain0" GEMM_EPI=res timeout -k 10 300 python -u scripts/gemm_bench.py $m@48 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r04w_gemm_ab.txt || exit 1
  done
done
o=gpurun_out/r04w_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py 48 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2; do
  run LS_GEMM_AREG=1 || exit 1
  run LS_GEMM_AREG=0 || exit 1
done
exit 0
