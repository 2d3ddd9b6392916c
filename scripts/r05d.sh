#!/bin/bash
# round 5: (1) halo convs with the GroupNorm affine input, new vs previous ls_gemm.hip;
# (2) whole-step 3-way: A new, C new with the N = 1280 linears back on 128x160
# (LS_GEMM_BIG1280=0), B previous source (libls_hip_ab.so); (3) PMC of the fused FeedForward
# and of the K = 320 residual row-block GEMM; (4) the per-call step table with roofline excess
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r05d_halo_ab.txt
S="conv0,conv1,vae conv 128 256,vae conv 256 128"
for r in 1 2; do
  GEMM_ONLY="$S" GEMM_EPI=aff,res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/A /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so GEMM_ONLY="$S" GEMM_EPI=aff,res timeout -k 10 200 python -u scripts/gemm_bench.py dma@48 2>&1 | grep -v amdgpu.ids | sed "s/^/B /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
o=gpurun_out/r05d_step_ab.txt
for r in 1 2; do
  timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/A$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_GEMM_BIG1280=0 timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/C$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 300 python -u scripts/step_ab.py 48 256 2>&1 | grep -v amdgpu.ids | sed "s/^/B$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS"
for pass in 1 2; do
  eval c=\$P$pass
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r05d_ff_p$pass -o run -- python3 scripts/ff_one.py 5 > gpurun_out/r05d_ff_p$pass.log 2>&1
  rc=$?; echo "ff pass$pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05d_ff_p$pass.log; exit $rc; }
done
python3 scripts/pmc_summary.py gpurun_out/r05d_ff_p1 gpurun_out/r05d_ff_p2 > gpurun_out/r05d_ff_pmc.txt; head -30 gpurun_out/r05d_ff_pmc.txt
SHAPE="786432 320 320 1 1" bash scripts/gemm_pmc.sh r05d_rb320 "0" > /dev/null || exit 1
head -30 gpurun_out/r05d_rb320_summary.txt
timeout -k 10 300 python -u scripts/step_calls.py 48 256 > gpurun_out/r05d_step_calls.txt 2>&1; rc=$?; head -45 gpurun_out/r05d_step_calls.txt; exit $rc
