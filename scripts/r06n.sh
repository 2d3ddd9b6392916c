#!/bin/bash
# round 6: ff_chain variants -- default (buffer DMA + bias-initialised accumulators), ab (global_load_lds
# DMA + bias-initialised), ab2 (buffer DMA + bias added late), ab3 (HEAD): kernel time
set -o pipefail
mkdir -p gpurun_out
o=gpurun_out/r06n_ab.txt
rm -f $o
for r in 1 2; do
  for v in default ab ab2 ab3; do
    if [ $v = default ]; then unset LS_HIP_LIB; else export LS_HIP_LIB=latentsync_amd/libls_hip_$v.so; fi
    timeout -k 10 300 python -u scripts/ff_chain_bench.py 2>&1 | grep -v amdgpu.ids | grep "ls_ff_chain" | sed "s/^/$v-$r /" | tee -a $o; rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
