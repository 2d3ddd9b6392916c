# usage: bash scripts/microbench.sh "<gemm modes>" [attn]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gemm_bench.py $1 > gpurun_out/gemm.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/gemm.log; [ $rc -ne 0 ] && exit $rc
if [ "$2" = attn ]; then timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/attn.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/attn.log; fi
exit $rc
