#!/bin/bash
# round 4: new-kernel tests first, then the whole GPU suite, the bench, and a kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04d}
timeout -k 10 400 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_ops.py -x -q -m gpu -k "halo or cross or attention" --timeout 200 --timeout-method thread > gpurun_out/${T}_new_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_new_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "not headline" --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-single-window --no-whisper > gpurun_out/${T}_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/${T}_prof -name "*kernel_trace.csv" | head -1)
python3 scripts/step_breakdown.py $f 30 > gpurun_out/${T}_step_breakdown.txt 2>&1
python3 scripts/phase_breakdown.py $f > gpurun_out/${T}_phase_breakdown.txt 2>&1
s=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp $s gpurun_out/${T}_kernel_stats.csv
head -25 gpurun_out/${T}_step_breakdown.txt
exit 0
