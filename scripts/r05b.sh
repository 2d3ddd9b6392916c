#!/bin/bash
# round 5: default build without the diagnostic kernels -- GPU tests (non-headline), the new
# configs[2] 16-frame window, and 256x256 vs 128x160 tiles on the N = 1280 1x1 shapes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "not headline" --timeout 200 --timeout-method thread > gpurun_out/r05b_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r05b_tests.log; [ $rc -ne 0 ] && exit $rc
grep -h "served window\|engine of 16\|bucketed engine" gpurun_out/r05b_tests.log
o=gpurun_out/r05b_n1280.txt
for r in 1 2; do
  for mode in dma t5 t9; do
    GEMM_ONLY="out2,sc2,out3,ff2_2,ff2_3,sc3" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py $mode@48 2>&1 | grep -v amdgpu.ids | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -s -q -m gpu -k "headline and 16-10" --timeout 500 --timeout-method thread > gpurun_out/r05b_headline.log 2>&1; rc=$?; grep -E "headline-depth|per-pixel|passed|failed" gpurun_out/r05b_headline.log; exit $rc
