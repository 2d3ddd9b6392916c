#!/bin/bash
# re-check of the fusion defaults on the final tree: fused FeedForward / temporal attention
# off vs on, same box, 48 windows
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r04z_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py 48 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2; do
  run LS_NOTHING=1 || exit 1
  run LS_FUSED_FF=0 || exit 1
  run LS_FUSED_TEMPORAL=0 || exit 1
done
exit 0
