#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each) over one GEMM shape (scripts/gemm_one.py),
# per forced tile.  usage: SHAPE="M K N ks res" bash scripts/gemm_pmc.sh TAG "TILES"
# -> gpurun_out/TAG_t<tile>_p<pass>; summary: python scripts/pmc_summary.py gpurun_out/TAG_*
set -o pipefail
tag=${1:-gpmc}
tiles=${2:-"0"}
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
P4="SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_WAIT_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_ACTIVE_INST_SCA SQ_IFETCH"
for t in $tiles; do
  for pass in 1 2 3 4; do
    eval c=\$P$pass
    TILE=$t REPS=10 timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${tag}_t${t}_p$pass -o run -- python3 scripts/gemm_one.py > gpurun_out/${tag}_t${t}_p$pass.log 2>&1
    rc=$?; echo "tile $t pass$pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${tag}_t${t}_p$pass.log; exit $rc; }
  done
done
python3 scripts/pmc_summary.py gpurun_out/${tag}_t* > gpurun_out/${tag}_summary.txt; rc=$?
cat gpurun_out/${tag}_summary.txt
exit $rc
