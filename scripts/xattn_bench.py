"""Time (HIP events, graph of 10) the fused audio cross-attention block at the bench's
48-window 32x32 level (M = 786432 rows, 50 tokens) -- PMC target.  usage: python
scripts/xattn_bench.py [windows] [reps]"""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from latentsync_amd import ops

nw = int(sys.argv[1]) if len(sys.argv) > 1 else 48
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
C, H, L, hw = 320, 8, 50, 1024
n_img = 16 * nw
M = n_img * hw
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(5)
r = lambda *s, sc=1.0: torch.randn(*s, generator=g) * sc
x = (r(M, C) * 1.5).to(torch.bfloat16).to(dev)
kv = r(n_img * L, 2 * C).to(torch.bfloat16).to(dev)
pk = ops.pack_cross_attention(r(C, C, sc=C ** -0.5), 1 + 0.1 * r(C), 0.1 * r(C), r(C, C, sc=C ** -0.5), 0.1 * r(C), H, dev)
st = ops.row_stats(x)
st2 = torch.empty_like(st)
out = torch.empty_like(x)
launch = lambda: ops.cross_attention_block(x, st, pk, kv, L, hw, st2, out=out)
launch()
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); launch(); e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
fl = 2.0 * M * C * C * 2 + 4.0 * M * H * L * (C // H)
print(f"xattn fused M={M} L={L}: {statistics.median(ts):.1f} us  ({fl / statistics.median(ts) / 1e6:.1f} TF/s algorithmic)")
