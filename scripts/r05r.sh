#!/bin/bash
# round 5: GroupNorm slot-sum finalize with 4 slots' loads in flight per thread vs the
# previous loop (libls_hip_ab.so): GN tests, whole step + VAE
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "gn or groupnorm" -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05r_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05r_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r05r_step_ab.txt
rm -f $o
for r in 1 2 3; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/new-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/old-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
