set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python3 -c "
import sys; sys.path.insert(0, '.')
from latentsync_amd import _lib
lib = _lib.load()
print('gemm occupancy (WG/CU): 128x160', lib.ls_gemm_occupancy(1), ' 256x256', lib.ls_gemm_occupancy(2), ' 128x128', lib.ls_gemm_occupancy(3))
" > gpurun_out/p5_gemm.log 2>&1
timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 >> gpurun_out/p5_gemm.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/step_calls.py 8 > gpurun_out/p5_calls.log 2>&1
