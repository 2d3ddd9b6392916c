#!/bin/bash
# round 6: UNet conv_norm_out + SiLU + conv_out on the narrow halo tile (default) vs the materialised
# GroupNorm + 4-column tiled GEMM (LS_NARROW_OUT=0, diagnostics mode): parity, step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_pipeline.py tests/test_gpu_bench_config.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06r_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r06r_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r06r_ab.txt
rm -f $o
for r in 1 2 3; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/narrow-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_DIAG_BUILD=1 LS_NARROW_OUT=0 timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/gnapply-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
