# attention micro-bench at 32 windows: default dispatch vs LS_ATTN_V1 (16-query kernel) -- small shapes
export NO_SDPA=1 WINDOWS=32
timeout -k 10 200 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
LS_ATTN_V1=1 timeout -k 10 200 python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu.ids
