#!/bin/bash
# round 6: per-call table of one 48-window step + encode / decode phases on the current tree
set -o pipefail
mkdir -p gpurun_out
for ph in step encode decode; do
  timeout -k 10 300 python -u scripts/step_calls.py 48 256 $ph > gpurun_out/r06e_${ph}_calls.txt 2>&1; rc=$?; head -14 gpurun_out/r06e_${ph}_calls.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
