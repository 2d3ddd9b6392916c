#!/bin/bash
# Build the library with extra device-compiler flags into latentsync_amd/libls_hip_<tag>.so,
# reporting VGPR spills per kernel (the product build refuses spills in counted-vmcnt kernels)
# usage: bash scripts/build_flags_ab.sh TAG "FLAGS"
set -e
tag=$1; flags=$2
root=$(cd "$(dirname "$0")/.." && pwd)
ab=$root/build/ab_$tag
rm -rf "$ab" && mkdir -p "$ab"
cd "$root/latentsync_amd/csrc"
pids=()
for f in *.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -munsafe-fp-atomics \
    -fno-slp-vectorize $flags -Rpass-analysis=kernel-resource-usage -c "$f" -o "$ab/${f%.hip}.o" 2> "$ab/${f%.hip}.rem" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p" || { echo "a compile failed (see $ab/*.rem)"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/latentsync_amd/libls_hip_$tag.so" "$ab"/*.o
python3 - "$ab" <<'PY'
import glob, re, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.rem")):
    name = None
    for line in open(f):
        m = re.search(r"Function Name: (\S+)", line)
        if m: name = m.group(1)
        m = re.search(r"VGPRs Spill: (\d+)", line)
        if m and int(m.group(1)) and name: print("spill", m.group(1), name[:90])
PY
echo "built latentsync_amd/libls_hip_$tag.so ($flags)"
