#!/bin/bash
# row-block GEMM: accumulators start at the bias, row statistics by bf16 dot2 -- vs HEAD
# (libls_hip_ab.so), same box: GPU tests, row-block shapes, step A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread -k "not headline" > gpurun_out/r04r_gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r04r_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r04r_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py 48 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2 3; do
  run LS_NOTHING=1 || exit 1
  run LS_HIP_LIB=latentsync_amd/libls_hip_ab.so || exit 1
done
exit 0
