"""Kernel time of ls_ff_chain (rows per wave 32 / 16) against the three launches it replaces
(to_out row-block GEMM with row statistics, ls_feedforward, proj_out with GroupNorm column
sums) at the bench's 32x32 level (48 windows: M = 786432, C = 320).
usage: python scripts/ff_chain_bench.py [M]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from latentsync_amd import _lib, ops  # noqa: E402
from latentsync_amd.packing import pack_ff_w2  # noqa: E402
from latentsync_amd.unet import _Dev, _ff  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 786432
C, I = 320, 1280
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
r = lambda *s, sc=1.0: torch.randn(*s, generator=g) * sc
bf = lambda t: t.to(torch.bfloat16).to(dev)
o, h1, xb = bf(r(M, C)), bf(r(M, C)), bf(r(M, C))
dv = _Dev({"wo": r(C, C, sc=C ** -0.5), "bo": r(C, sc=0.1), "w2": r(C, I, sc=I ** -0.5), "b2": r(C, sc=0.1),
           "wp": r(C, C, sc=C ** -0.5), "bp": r(C, sc=0.1)}, dev)
pko, pkp, ff2 = dv.packed("wo", "bo"), dv.packed("wp", "bp"), dv.packed("w2", "b2")
ff1 = dv.packed_ln(r(2 * I, C, sc=C ** -0.5), r(2 * I, sc=0.1), (1 + 0.1 * r(C), 0.1 * r(C)), geglu=True)
ff2p = pack_ff_w2(dv.sd["w2"].float()).to(torch.bfloat16).to(dev)
chain = ops.pack_ff_chain(pko, ff1, ff2, pkp)
lib = _lib.load()
st = torch.empty((M, 2), dtype=torch.float32, device=dev)


def unfused():
    h2 = ops.linear(o, pko, res=h1, stats_out=st)
    y = ops.feedforward(h2, st, ff1, ff2, ff2p)
    return ops.conv(y.view(1, 1, M, C), pkp, res=xb.view(1, 1, M, C), gn_out=True)


def timed(fn, n=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[n // 2]


fl = 4.0 * M * C * C + 6.0 * M * C * I
for fmr in (1, 2):
    if lib.ls_set_tuning(17, fmr) != 0:
        continue  # 32 rows per wave: diagnostics build only
    t = timed(lambda: ops.ff_chain(o, h1, xb, chain))
    print(f"ls_ff_chain M={M} rows/wave {16 * fmr}: {t:.1f} us, {fl / t / 1e6:.1f} TF/s")
lib.ls_set_tuning(17, 1)
t = timed(unfused)
print(f"unfused (to_out + ls_feedforward + proj_out) M={M}: {t:.1f} us, {fl / t / 1e6:.1f} TF/s")
t = timed(lambda: ops.feedforward(h1, st, ff1, ff2, ff2p))
print(f"  of which ls_feedforward: {t:.1f} us")
