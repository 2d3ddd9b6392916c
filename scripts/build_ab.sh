#!/bin/bash
# Build an A/B variant of libls_hip.so: the current sources with ONE file taken from
# another commit, written to latentsync_amd/libls_hip_ab.so (select it at run time
# with LS_HIP_LIB=latentsync_amd/libls_hip_ab.so).
# usage: bash scripts/build_ab.sh COMMIT [csrc file(s), default ls_gemm.hip]
#        COMMIT "-" = the working tree's file; EXTRA_FLAGS (env) adds hipcc flags (-DMACRO=...);
#        AB_OUT (env) names the output library (default latentsync_amd/libls_hip_ab.so)
set -e
commit=$1; shift; files=${*:-ls_gemm.hip}
root=$(cd "$(dirname "$0")/.." && pwd)
out=${AB_OUT:-latentsync_amd/libls_hip_ab.so}
ab=$root/build/ab
rm -rf "$ab" && mkdir -p "$ab/latentsync_amd/csrc" "$ab/include"
cp "$root/include/ls_hip.h" "$ab/include/"
cp "$root"/latentsync_amd/csrc/* "$ab/latentsync_amd/csrc/"
if [ "$commit" != "-" ]; then
  for file in $files; do git -C "$root" show "$commit:latentsync_amd/csrc/$file" > "$ab/latentsync_amd/csrc/$file"; done
fi
cd "$ab/latentsync_amd/csrc"
pids=()
for f in *.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -munsafe-fp-atomics \
    -fno-slp-vectorize $EXTRA_FLAGS -c "$f" -o "${f%.hip}.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p" || { echo "a compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/$out" *.o
echo "built $out ($files from $commit, extra flags: ${EXTRA_FLAGS:-none})"
