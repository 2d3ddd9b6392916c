# temporal attention 16-B stores: parity tests, micro-bench, smoke
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py -k "attention or motion" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
NO_SDPA=1 WINDOWS=32 ATTN_ONLY=temporal timeout -k 10 100 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" 2>&1 | tail -2
