# Two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE -- separate runs, TCC slots) of a
# short eager bench, then the per-ls_conv2d-call HBM traffic -> profiles/pmc_traffic.json
# usage: bash scripts/pmc_pass.sh TAG [windows per UNet call, default 48 = bench.py's configs[1]]
set -o pipefail
tag=${1:-pmc}
nw=${2:-48}
export TMPDIR=/tmp
mkdir -p gpurun_out
B="scripts/pmc_step.py $nw 3"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${tag}_$c -o run -- python3 $B > gpurun_out/${tag}_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${tag}_$c.log; exit $rc; }
done
python3 scripts/pmc_traffic.py gpurun_out/${tag}_FETCH_SIZE gpurun_out/${tag}_WRITE_SIZE gpurun_out/${tag}_traffic.json
python3 scripts/pmc_per_kernel.py gpurun_out/${tag}_FETCH_SIZE gpurun_out/${tag}_WRITE_SIZE 60 > gpurun_out/${tag}_per_kernel.txt
