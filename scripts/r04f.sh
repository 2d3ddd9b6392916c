#!/bin/bash
# round 4: the GPU suite, the bench, a kernel trace, then the r04e A/Bs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04f}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "not headline" --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_bench.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-single-window --no-whisper > gpurun_out/${T}_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/${T}_prof -name "*kernel_trace.csv" | head -1)
python3 scripts/step_breakdown.py $f 30 > gpurun_out/${T}_step_breakdown.txt 2>&1
python3 scripts/phase_breakdown.py $f > gpurun_out/${T}_phase_breakdown.txt 2>&1
s=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp $s gpurun_out/${T}_kernel_stats.csv
rm -rf gpurun_out/${T}_prof
head -12 gpurun_out/${T}_step_breakdown.txt
timeout -k 10 500 bash scripts/r04e.sh > gpurun_out/${T}_r04e.log 2>&1; rc=$?; tail -4 gpurun_out/r04e_ab.txt; exit $rc
