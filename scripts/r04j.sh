#!/bin/bash
# same-box step / encode / decode A/Bs at 48 windows (two alternations each):
# fused audio cross-attention block vs q GEMM + SDPA + out GEMM; halo conv vs tiled conv
# behind a materialised GroupNorm; halo pieces over the read pixels (RP) vs the padded image
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r04j_step_ab.txt
run() { echo "== $*" | tee -a $o; env "$@" timeout -k 10 300 python -u scripts/step_ab.py 48 2>&1 | grep -v amdgpu.ids | tee -a $o; }
for r in 1 2; do
  run LS_FUSED_XATTN=1 || exit 1
  run LS_FUSED_XATTN=0 || exit 1
  run LS_HALO=0 || exit 1
  run LS_HALO_RP=1 || exit 1
done
exit 0
