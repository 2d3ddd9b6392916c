#!/bin/bash
# K = 640 residual GEMMs on the row-block kernel too (LS_GEMM_RB640_RES=1) now that K = 640
# row blocks take two fragments per wave: step A/B, same box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r04y_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py 48 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2; do
  run LS_GEMM_RB640_RES=1 || exit 1
  run LS_NOTHING=1 || exit 1
done
exit 0
