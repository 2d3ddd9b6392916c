#!/bin/bash
# round 6: ls_ff_chain parity + UNet goldens + 48-window parity, then the step A/B (chain on / off)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "ff_chain or feedforward or rowblock640_affine" tests/test_gpu_unet.py tests/test_gpu_blocks.py tests/test_gpu_bench_config.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r06b_tests.log 2>&1; rc=$?; grep -E "rel|passed|failed|Error" gpurun_out/r06b_tests.log | tail -30; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r06b_step_ab.txt
rm -f $o
for r in 1 2 3; do
  for c in 1 0; do
    LS_DIAG_BUILD=1 LS_FF_CHAIN=$c timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/chain=$c-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
