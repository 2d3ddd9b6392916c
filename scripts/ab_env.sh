#!/bin/bash
# Same-box A/B of one environment switch on a short bench under rocprofv3 --kernel-trace,
# alternated (A, B, A, B).  A = plain run, B = with "$2" (e.g. LS_GEMM_GLDS=1) exported.
# Comparison (scripts/cmp_steps.py, per-kernel minimum over the runs) -> gpurun_out/TAG_cmp.txt.
# usage: bash scripts/ab_env.sh TAG "VAR=VALUE"
set -o pipefail
tag=${1:-abenv}
envb=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in A B; do
    if [ $v = B ]; then e="env $envb"; else e=""; fi
    ( [ $v = B ] && export $envb; timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${tag}_${v}$r -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-single-window --no-whisper > gpurun_out/${tag}_${v}$r.log 2>&1 )
    rc=$?; echo "$v$r rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
python3 scripts/cmp_steps.py "gpurun_out/${tag}_A*" "gpurun_out/${tag}_B*" 20 > gpurun_out/${tag}_cmp.txt
rc=$?; cat gpurun_out/${tag}_cmp.txt
rm -rf gpurun_out/${tag}_A? gpurun_out/${tag}_B?
exit $rc
