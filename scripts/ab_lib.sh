#!/bin/bash
# Same-box A/B of two library builds on a short bench under rocprofv3 --kernel-trace:
# the shipped latentsync_amd/libls_hip.so and LS_HIP_LIB=latentsync_amd/libls_hip_ab.so,
# alternated (shipped, ab, shipped, ab) so drift (clocks, temperature) hits both.
# The comparison (scripts/cmp_steps.py, per-kernel minimum over the runs) -> gpurun_out/TAG_cmp.txt.
# usage: bash scripts/ab_lib.sh TAG
set -o pipefail
tag=${1:-ablib}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in shipped ab; do
    lib=latentsync_amd/libls_hip.so; [ $v = ab ] && lib=latentsync_amd/libls_hip_ab.so
    LS_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${tag}_${v}$r -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-single-window --no-whisper > gpurun_out/${tag}_${v}$r.log 2>&1
    rc=$?; echo "$v$r rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
python3 scripts/cmp_steps.py "gpurun_out/${tag}_shipped*" "gpurun_out/${tag}_ab*" 16 > gpurun_out/${tag}_cmp.txt
rc=$?; cat gpurun_out/${tag}_cmp.txt
rm -rf gpurun_out/${tag}_shipped? gpurun_out/${tag}_ab?  # traces stay on the box (the copy-back cap)
exit $rc
