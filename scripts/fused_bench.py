"""Micro-bench of the fused motion attention (ls_temporal_attention) against the
unfused launches it replaces, at the UNet's 32x32 / 16x16 level shapes and the bench's
window count (HIP events on the launch stream, median of 20 after warm-up).

    python scripts/fused_bench.py [windows]
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from latentsync_amd import ops  # noqa: E402
from latentsync_amd.unet import _Dev, positional_encoding  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[n // 2]


def main():
    nw = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    dv = _Dev({}, dev)
    only = os.environ.get("ONLY", "")
    for C, S in ((320, 1024), (640, 256)):
        if only and only != "attn":
            break
        B, Fr = nw, 16
        M = B * Fr * S
        d = C // 8
        x = torch.randn((M, C), generator=g).to(torch.bfloat16).to(dev)
        wq, wk, wv = (torch.randn((C, C), generator=g) / math.sqrt(C) for _ in range(3))
        gamma, beta = 1 + 0.1 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
        pe = positional_encoding(C, 24)
        pk = ops.pack_temporal(wq, wk, wv, gamma, beta, pe, 8, dev)
        o = torch.empty_like(x)
        t_f = timeit(lambda: ops.temporal_attention(x, pk, B, Fr, S, out=o))
        pq = dv.packed_ln(torch.cat([wq, wk, wv]), None, (gamma, beta), pe=pe)
        st = ops.row_stats(x)
        rv = (pq.pe_rows, S, pq.pe_rows.shape[1], Fr)
        qkv = ops.linear(x, pq, ln_stats=st, rowvec=rv)
        t_g = timeit(lambda: ops.linear(x, pq, ln_stats=st, rowvec=rv, out=qkv.view(1, 1, M, 3 * C)))
        sst = (Fr * S * 3 * C, 3 * C, S * 3 * C, d)
        t_a = timeit(lambda: ops.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=B * S, z2=S, heads=8, nq=Fr,
                                           nk=Fr, head_dim=d, qs=sst, ks=sst, vs=sst, os_=(Fr * S * C, C, S * C, d)))
        fl = 2.0 * M * 3 * C * C + 4.0 * B * S * 8 * Fr * Fr * d
        print(f"temporal C={C} M={M}: fused {t_f:8.1f} us ({fl / t_f / 1e6:6.1f} TF/s)   "
              f"qkv GEMM {t_g:8.1f} + attention {t_a:7.1f} = {t_g + t_a:8.1f} us")


if __name__ == "__main__":
    main()
