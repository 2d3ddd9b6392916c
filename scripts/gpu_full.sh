#!/bin/bash
# GPU-box round check: gpu tests -> bench (default config) -> rocprofv3 kernel stats of a short bench.
# Stops at the first failure; every GPU step has its own time limit.
# usage: bash scripts/gpu_full.sh TAG [bench args...]
set -o pipefail
tag=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/${tag}_tests.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${tag}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/${tag}_bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-single-window "$@" > gpurun_out/${tag}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/${tag}_prof.log
exit $rc
