#!/bin/bash
# round 5 checkpoint: the bench (no CPU leg) and a kernel trace with step / phase breakdowns
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05i}
timeout -k 10 500 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d gpurun_out/${T}_prof -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-single-window --no-whisper > gpurun_out/${T}_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/${T}_prof -name "*kernel_trace.csv" | head -1)
python3 scripts/step_breakdown.py $f 40 > gpurun_out/${T}_step_breakdown.txt 2>&1
db=$(find gpurun_out/${T}_prof -name "*.db" | head -1)
python3 scripts/phase_breakdown.py $db > gpurun_out/${T}_phase_breakdown.txt 2>&1
s=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp $s gpurun_out/${T}_kernel_stats.csv
rm -rf gpurun_out/${T}_prof
head -24 gpurun_out/${T}_step_breakdown.txt
cat gpurun_out/${T}_phase_breakdown.txt | head -20
exit 0
