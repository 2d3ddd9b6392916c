#!/bin/bash
# round 6 final tree (after the column-sum change), part B: PMC traffic (first, so the bench line carries it), the headline
# bench with its CPU baseline, kernel trace + step / phase breakdowns, per-call tables, serving
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06x
bash scripts/pmc_pass.sh ${T}_pmc 48 || exit 1
cp gpurun_out/${T}_pmc_traffic.json profiles/pmc_traffic.json
rm -rf gpurun_out/${T}_pmc_FETCH_SIZE gpurun_out/${T}_pmc_WRITE_SIZE
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_bench.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d gpurun_out/${T}_prof -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-single-window --no-whisper > gpurun_out/${T}_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/${T}_prof -name "*kernel_trace.csv" | head -1)
python3 scripts/step_breakdown.py $f 40 > gpurun_out/${T}_step_breakdown.txt 2>&1
db=$(find gpurun_out/${T}_prof -name "*.db" | head -1)
python3 scripts/phase_breakdown.py $db > gpurun_out/${T}_phase_breakdown.txt 2>&1
s=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp $s gpurun_out/${T}_kernel_stats.csv
rm -rf gpurun_out/${T}_prof
head -12 gpurun_out/${T}_step_breakdown.txt
head -4 gpurun_out/${T}_phase_breakdown.txt
for ph in step encode decode; do
  timeout -k 10 300 python -u scripts/step_calls.py 48 256 $ph > gpurun_out/${T}_${ph}_calls.txt 2>&1; rc=$?; echo "step_calls $ph rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 python -u scripts/serve_latency.py 2>&1 | grep -v amdgpu.ids > gpurun_out/${T}_serve_latency.txt; rc=$?; tail -8 gpurun_out/${T}_serve_latency.txt; exit $rc
