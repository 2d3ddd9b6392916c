# Two PMC passes (SQ counters) over scripts/fused_bench.py: the fused temporal attention
# kernel and the q|k|v row-block GEMM it replaces.  usage: bash scripts/fused_pmc.sh TAG
set -o pipefail
tag=${1:-fpmc}
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS"
for pass in 1 2; do
  eval c=\$P$pass
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${tag}_p$pass -o run -- python3 scripts/fused_bench.py 8 > gpurun_out/${tag}_p$pass.log 2>&1
  rc=$?; echo "pass$pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${tag}_p$pass.log; exit $rc; }
done
python3 scripts/pmc_summary.py gpurun_out/${tag}_p1 gpurun_out/${tag}_p2 > gpurun_out/${tag}_summary.txt
cat gpurun_out/${tag}_summary.txt
