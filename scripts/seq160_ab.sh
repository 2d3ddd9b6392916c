# d = 160 temporal attention on MFMA (head-split seqm): attention parity tests + micro-bench A/B
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k "attention" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
export NO_SDPA=1 WINDOWS=32 ATTN_ONLY=temporal
timeout -k 10 100 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu || exit 1
LS_ATTN_SEQ160_VALU=1 timeout -k 10 100 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu
LS_ATTN_SEQ_HS2=1 timeout -k 10 100 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu | sed 's/^/hs2 /'
LS_ATTN_SEQ_HS2=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k "temporal" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
