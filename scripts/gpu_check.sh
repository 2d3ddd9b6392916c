#!/bin/bash
# GPU-box check: gpu tests, then a bench line; stops on any crash / timeout.
# usage: bash scripts/gpu_check.sh [tag] [bench args...]
tag=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -q -m gpu -s > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "rel_err|passed|failed" gpurun_out/${tag}_tests.log | tail -25
if [ $rc -gt 1 ]; then echo "pytest crashed/timed out: stopping"; exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/${tag}_bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/${tag}_bench.log
exit $rc
