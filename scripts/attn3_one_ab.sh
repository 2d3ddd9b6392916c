# single-tile attn3 (nk <= 64): attention parity tests + micro-bench A/B (LS_ATTN3_TWO_STAGE=1 = old)
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k "attention" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
export NO_SDPA=1 WINDOWS=32
for v in new old; do
  e=""; [ $v = old ] && e="LS_ATTN3_TWO_STAGE=1"
  for o in cross "spatial L2" "spatial L3"; do
    env $e ATTN_ONLY="$o" timeout -k 10 100 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 1
  done
done
