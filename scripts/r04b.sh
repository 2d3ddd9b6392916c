#!/bin/bash
# round 4, first GPU pass: attention parity, attn6 vs attn5 A/B, 48-window per-call table,
# then the full final check (tests, headline-depth windows, smoke, bench)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "attention or cross" --timeout 120 --timeout-method thread > gpurun_out/r04b_attn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r04b_attn_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in A B; do
    if [ $v = B ]; then e="LS_ATTN5=1"; else e="LS_NONE=1"; fi
    env $e WINDOWS=48 ATTN_ONLY="spatial L0" NO_SDPA=1 timeout -k 10 200 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v$r /" | tee -a gpurun_out/r04b_attn_ab.txt; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 300 python -u scripts/step_calls.py 48 256 > gpurun_out/r04b_step_calls_w48.txt 2>&1; rc=$?; head -40 gpurun_out/r04b_step_calls_w48.txt; [ $rc -ne 0 ] && exit $rc
ROUNDS=1 timeout -k 10 400 bash scripts/r04c.sh > gpurun_out/r04c.log 2>&1; rc=$?; tail -3 gpurun_out/r04c.log; [ $rc -ne 0 ] && exit $rc
SKIP_HEADLINE=1 TAG=r04b bash scripts/final_check.sh
