# attn3 (single tile) 16-B output stores: attention parity tests + micro-bench (new vs HEAD's ls_attn.hip)
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py tests/test_gpu_unet.py -k "attention or transformer or unet" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
export NO_SDPA=1 WINDOWS=32
for r in 1 2; do
  for o in cross "spatial L2"; do
    ATTN_ONLY="$o" timeout -k 10 100 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu | sed "s/^/new /" || exit 1
    ATTN_ONLY="$o" LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 100 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu | sed "s/^/old /" || exit 1
  done
done
