#!/bin/bash
# round 5: epilogue residual prefetch (last K-tile / one pass ahead) + row-block residual
# retired a chunk later.  GPU tests on the new build, then same-box GEMM A/B against the
# previous ls_gemm.hip (libls_hip_ab.so), then the N = 1280 tile sweep
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "not headline" --timeout 200 --timeout-method thread > gpurun_out/r05c_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r05c_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -m pytest tests/test_gpu_pipeline.py -x -q -s -m gpu -k "share_one_engine" --timeout 150 --timeout-method thread 2>&1 | grep -E "engine of|bucketed|passed|failed"
o=gpurun_out/r05c_epi_ab.txt
S="out0,out1,out2,ff2_0,ff2_1,ff2_2,conv0,conv1,vae conv 128 256"
for r in 1 2; do
  GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/A /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so GEMM_ONLY="$S" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/B /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
o=gpurun_out/r05c_n1280.txt
for mode in dma t5 t9; do
  GEMM_ONLY="out2,sc2,out3,ff2_2,ff2_3,sc3" GEMM_EPI=res timeout -k 10 200 python -u scripts/gemm_bench.py $mode@48 2>&1 | grep -v amdgpu.ids | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
