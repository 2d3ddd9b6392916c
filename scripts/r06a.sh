#!/bin/bash
# round 6: the new parity tests (48-window UNet / engine, timestep forms) + a bench line with memory
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_unet.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r06a_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06a_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r06a_bench.log 2>&1; rc=$?; tail -1 gpurun_out/r06a_bench.log | cut -c1-300; exit $rc
