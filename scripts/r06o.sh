#!/bin/bash
# round 6: buffer-descriptor DMA in ff_chain, the row-block GEMM and the temporal attention (default) vs HEAD (ab lib)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "ff_chain or feedforward or layernorm_folded or rowblock or linear or gemm or temporal or tattn" -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r06o_tests.log 2>&1; rc=$?; grep -E "rel|passed|failed|Error" gpurun_out/r06o_tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_blocks.py tests/test_gpu_temporal.py tests/test_gpu_bench_config.py -x -q --timeout 300 --timeout-method thread >> gpurun_out/r06o_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06o_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r06o_ab.txt
rm -f $o
for r in 1 2; do
  timeout -k 10 300 python -u scripts/ff_chain_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/new-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/ff_chain_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/head-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2 3; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/new-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/head-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
