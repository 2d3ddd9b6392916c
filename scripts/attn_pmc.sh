# PMC passes over the d=40 spatial attention kernel variants (scripts/attn_bench.py,
# 16 windows).  usage: bash scripts/attn_pmc.sh TAG  -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-apmc}
export TMPDIR=/tmp ATTN_ONLY="spatial L0" WINDOWS=16 NO_SDPA=1
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS"
for v in 0 3; do
  for pass in 1 2; do
    eval c=\$P$pass
    LS_ATTN_V4=$v timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${tag}_v${v}_p$pass -o run -- python3 scripts/attn_bench.py > gpurun_out/${tag}_v${v}_p$pass.log 2>&1
    rc=$?; echo "v$v pass$pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${tag}_v${v}_p$pass.log; exit $rc; }
  done
done
exit 0
