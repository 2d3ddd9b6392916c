#!/bin/bash
# round 6: narrow 16-column halo tile (VAE conv_out with conv_norm_out + SiLU fused): parity, VAE /
# pipeline against the oracle, decode / encode A/B (tuning key 19); then the GELU A/B (r06i.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r06j_tests.log 2>&1; rc=$?; grep -E "rel|passed|failed|Error" gpurun_out/r06j_tests.log | tail -16; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -k "vae_full_width" -x -v -s --timeout 300 --timeout-method thread >> gpurun_out/r06j_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06j_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -k "window_matches_oracle or run_windows_batches" -x -v -s --timeout 300 --timeout-method thread >> gpurun_out/r06j_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06j_tests.log; [ $rc -ne 0 ] && exit $rc
o=gpurun_out/r06j_ab.txt
rm -f $o
for r in 1 2; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/narrow-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_DIAG_BUILD=1 LS_TUNE=19=0 timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/tiled-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
bash scripts/r06i.sh
