#!/bin/bash
# PMC (two SQ passes) and timing of the fused audio cross-attention block
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/xattn_bench.py 48 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04u_xattn_time.txt || exit 1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS"
for pass in 1 2; do
  eval c=\$P$pass
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r04u_p$pass -o run -- python3 scripts/xattn_bench.py 48 4 > gpurun_out/r04u_p$pass.log 2>&1
  rc=$?; echo "pass$pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04u_p$pass.log; exit $rc; }
done
python3 scripts/pmc_summary.py gpurun_out/r04u_p1 gpurun_out/r04u_p2 > gpurun_out/r04u_summary.txt; cat gpurun_out/r04u_summary.txt
