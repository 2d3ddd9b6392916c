#!/bin/bash
# K = 640 row-block GEMM with two fragments per wave (LS_RB640_FM2: 256-row blocks) vs one:
# GPU tests under the switch, step / encode / decode A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LS_RB640_FM2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py tests/test_gpu_unet.py tests/test_gpu_temporal.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04x_gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r04x_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r04x_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py 48 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2 3; do
  run LS_RB640_FM2=1 || exit 1
  run LS_NOTHING=1 || exit 1
done
exit 0
