#!/bin/bash
# PMC passes on the final kernels: the halo conv (UNet 320 ch at 32^2, GN affine) and the
# fused FeedForward / temporal attention (scripts/fused_bench.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SHAPE="262144 2880 320 3 1" AFF=1 bash scripts/gemm_pmc.sh r04s_h320 "0" || exit 1
bash scripts/fused_pmc.sh r04s_fused || exit 1
exit 0
