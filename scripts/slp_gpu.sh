#!/bin/bash
# GPU half of the SLP investigation: scripts/slp_check.py on the shipped library and
# on each scripts/slp_variants.py build.  usage: bash scripts/slp_gpu.sh TAG
set -o pipefail
tag=${1:-slp}
mkdir -p gpurun_out
for v in ${VARIANTS:-"" slp slp_bw slp_sb}; do
  lib=latentsync_amd/libls_hip${v:+_$v}.so
  LS_HIP_LIB=$lib timeout -k 10 240 python -u scripts/slp_check.py 16 > gpurun_out/${tag}_${v:-shipped}.log 2>&1
  rc=$?; echo "${v:-shipped} rc=$rc: $(tail -1 gpurun_out/${tag}_${v:-shipped}.log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
