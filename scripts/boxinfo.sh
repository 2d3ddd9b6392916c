# one-line-per-fact description of the GPU box (clocks, power cap, CUs, LDS)
(rocm-smi --showclocks --showpower --showmaxpower --showperflevel --showuse 2>/dev/null | grep -v "^=\|^$" | head -30) || true
python3 - <<'PY'
import torch
p = torch.cuda.get_device_properties(0)
print("dev", p.name, "CUs", p.multi_processor_count, "gcn", getattr(p, "gcnArchName", "?"),
      "smem/blk", getattr(p, "shared_memory_per_block", "?"), "smem/mp", getattr(p, "shared_memory_per_multiprocessor", "?"),
      "L2", getattr(p, "L2_cache_size", "?"), "mem GB", p.total_memory / 2**30)
PY
env | grep -i "HSA_\|HIP_\|ROC\|GPU_" | grep -v PATH | sort
python3 -c "
import sys; sys.path.insert(0, '.')
from latentsync_amd import _lib
lib = _lib.load()
print('gemm occupancy (WG/CU): 128x160', lib.ls_gemm_occupancy(1), ' 256x256', lib.ls_gemm_occupancy(2), ' 128x128', lib.ls_gemm_occupancy(3))
"
