#!/bin/bash
# Same-box A/B of the GroupNorm producer statistics: rocprofv3 kernel traces of a short
# bench with LS_GN_EPILOGUE=0 (read-pass statistics) and =1.  usage: bash scripts/ab_gn.sh TAG
set -o pipefail
tag=${1:-abgn}
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
  LS_GN_EPILOGUE=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${tag}_$v -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-single-window --no-whisper > gpurun_out/${tag}_$v.log 2>&1
  rc=$?; echo "LS_GN_EPILOGUE=$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
