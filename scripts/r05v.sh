#!/bin/bash
# round 5: the headline bench itself, same box, grouped short-K raster on (default) vs off
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r05v_bench_ab.txt
rm -f $o
for r in 1 2; do
  for g in 1 0; do
    LS_GEMM_GM_SHORTK=$g timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-single-window --no-whisper > gpurun_out/r05v_b.log 2>&1; rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05v_b.log; exit $rc; }
    tail -1 gpurun_out/r05v_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gm4=$g-$r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a $o
  done
done
exit 0
