"""Run-to-run determinism of the attention kernels (bitwise) on the UNet shapes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from latentsync_amd import ops
for n, N, Nk, heads, d in [(16, 1024, 1024, 8, 40), (16, 256, 256, 8, 80), (16, 64, 64, 8, 160), (16, 1024, 50, 8, 40)]:
    C = heads * d
    q = torch.randn(n * N, C, device="cuda").to(torch.bfloat16)
    kv = torch.randn(n * Nk, 2 * C, device="cuda").to(torch.bfloat16)
    outs = []
    for _ in range(6):
        o = torch.empty_like(q)
        ops.attention(q, kv, kv[:, C:], o, batch=n, z2=1, heads=heads, nq=N, nk=Nk, head_dim=d,
                      qs=(N * C, 0, C, d), ks=(Nk * 2 * C, 0, 2 * C, d), vs=(Nk * 2 * C, 0, 2 * C, d),
                      os_=(N * C, 0, C, d))
        outs.append(o.clone())
    diffs = [int((o != outs[0]).sum()) for o in outs]
    print(f"attn n={n} N={N} Nk={Nk} d={d}: differing elements vs run0 {diffs}")
