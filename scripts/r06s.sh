#!/bin/bash
# round 6: 8-channel-input 3x3 conv (VAE conv_in; tuning key 22): parity, VAE / pipeline vs the oracle,
# encode / decode A/B against the tiled GEMM (LS_TUNE=22=0 in diagnostics mode)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -k "c8" -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r06s_tests.log 2>&1; rc=$?; grep -E "rel|passed|failed|Error" gpurun_out/r06s_tests.log | tail -6; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k "vae_full_width" tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread >> gpurun_out/r06s_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r06s_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r06s_ab.txt
rm -f $o
for r in 1 2 3; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/c8-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_DIAG_BUILD=1 LS_TUNE=22=0 timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/tiled-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
