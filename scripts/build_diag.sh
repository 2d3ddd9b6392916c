#!/bin/bash
# Diagnostic variant of libls_hip.so: the current sources with -D$1 (an ablation switch,
# e.g. LS_TATTN_ABLATE or LS_GEMM_ABLATE), written to latentsync_amd/libls_hip_ab.so --
# select it at run time with LS_HIP_LIB=latentsync_amd/libls_hip_ab.so.
# usage: bash scripts/build_diag.sh DEFINE
set -e
def=${1:?define}
root=$(cd "$(dirname "$0")/.." && pwd)
obj=$root/build/diag
mkdir -p "$obj"
objs=()
for f in "$root"/latentsync_amd/csrc/*.hip; do
  o=$obj/$(basename "${f%.hip}").o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -munsafe-fp-atomics \
    -fno-slp-vectorize -D"$def" -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/latentsync_amd/libls_hip_ab.so" "${objs[@]}"
echo "built latentsync_amd/libls_hip_ab.so with -D$def"
