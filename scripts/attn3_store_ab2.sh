# attn3 multi-tile 16-B stores: parity tests + micro-bench (new vs HEAD)
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py tests/test_gpu_unet.py tests/test_gpu_audio.py -k "attention or transformer or unet or whisper or encoder" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
export NO_SDPA=1 WINDOWS=32
for r in 1 2; do
  for o in "spatial L1" "spatial L2"; do
    ATTN_ONLY="$o" timeout -k 10 100 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu | sed "s/^/new /" || exit 1
    ATTN_ONLY="$o" LS_HIP_LIB=latentsync_amd/libls_hip_ab.so timeout -k 10 100 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu | sed "s/^/old /" || exit 1
  done
done
