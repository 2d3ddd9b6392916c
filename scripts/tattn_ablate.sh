# fused temporal attention ablation (diagnostic library, scripts/build_diag.sh -DLS_TATTN_ABLATE): which phase costs what
# usage (GPU box): bash scripts/tattn_ablate.sh
set -o pipefail
for v in 0 1 8 16 24 2 6 30; do
  LS_HIP_LIB=latentsync_amd/libls_hip_ab.so LS_TATTN_ABLATE=$v timeout -k 10 120 python -u scripts/fused_bench.py 32 2>&1 | grep temporal | sed "s/^/ablate $v: /" || exit 1
done
