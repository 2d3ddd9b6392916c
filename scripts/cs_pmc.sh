#!/bin/bash
# PMC passes over scripts/cs_cost.py (one shape): the halo conv with and without GroupNorm column sums
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-cspmc}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_SCA SQ_IFETCH SQ_ACTIVE_INST_MISC"
for pass in 1 2 3; do
  eval c=\$P$pass
  CS_ONLY="unet 32" timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${tag}_t0_p$pass -o run -- python3 scripts/cs_cost.py > gpurun_out/${tag}_p$pass.log 2>&1
  rc=$?; echo "pass$pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${tag}_p$pass.log; exit $rc; }
done
python3 scripts/pmc_summary.py gpurun_out/${tag}_t0_p* > gpurun_out/${tag}_summary.txt; rc=$?
cat gpurun_out/${tag}_summary.txt
exit $rc
