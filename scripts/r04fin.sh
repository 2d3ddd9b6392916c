#!/bin/bash
# final tree: bench + kernel trace (step / phase breakdowns, kernel stats), no headline tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04fin
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_bench.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d gpurun_out/${T}_prof -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-single-window --no-whisper > gpurun_out/${T}_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/${T}_prof -name "*kernel_trace.csv" | head -1)
python3 scripts/step_breakdown.py $f 30 > gpurun_out/${T}_step_breakdown.txt 2>&1
db=$(find gpurun_out/${T}_prof -name "*.db" | head -1)
python3 scripts/phase_breakdown.py $db > gpurun_out/${T}_phase_breakdown.txt 2>&1
s=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp $s gpurun_out/${T}_kernel_stats.csv
rm -rf gpurun_out/${T}_prof
head -20 gpurun_out/${T}_step_breakdown.txt
