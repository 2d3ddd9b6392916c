"""Cost of the GroupNorm column sums in the conv epilogue: one conv shape timed with and without
gn_out (the kernel's CSF instance vs the plain one), HIP events, median of 15 launches, the two
arms alternated three times (timing one arm first biased it: the chip had not reached its clock).
usage: python scripts/cs_cost.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from latentsync_amd import ops  # noqa: E402
from latentsync_amd.packing import pack_weight  # noqa: E402

dev = torch.device("cuda", 0)
SHAPES = [("unet 32^2 320->320 aff", 768, 32, 320, 320, True), ("unet 16^2 640->640 aff", 768, 16, 640, 640, True),
          ("vae 256^2 128->128 aff", 96, 256, 128, 128, True), ("vae 128^2 256->256 aff", 192, 128, 256, 256, True),
          ("unet 8^2 1280->1280 aff", 768, 8, 1280, 1280, True), ("unet 32^2 1x1 320->320", 768, 32, 320, 320, None),
          ("unet 16^2 1x1 640->640 +res", 768, 16, 640, 640, "res"),
          ("unet 8^2 1x1 1280->1280 +res", 768, 8, 1280, 1280, "res")]
SHAPES = [t for t in SHAPES if not os.environ.get("CS_ONLY") or any(o in t[0] for o in os.environ["CS_ONLY"].split(","))]


def timed(fn, n=15):
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


for name, n, H, cin, cout, aff in SHAPES:
    ks = 3 if aff is True else 1
    x = torch.randn(n, H, H, cin, device=dev).to(torch.bfloat16)
    w = torch.randn(cout, cin, ks, ks) / (cin * ks * ks) ** 0.5
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).to(dev), torch.zeros(cout, device=dev), cin, ks, cout)
    kw = {}
    if aff == "res":
        kw = dict(res=torch.randn(n, H, H, cout, device=dev).to(torch.bfloat16))
    elif aff:
        kw = dict(aff=(torch.rand(n, cin, device=dev) + 0.5, torch.randn(n, cin, device=dev) * 0.1, 1, True),
                  aff_materialize=True)
    out = torch.empty(n, H, H, cout, dtype=torch.bfloat16, device=dev)
    path = ops.conv_path(x, pw, **{k: v for k, v in kw.items() if k == "aff"})
    # alternated, three rounds each (the first-measured arm had run at a lower clock)
    f1 = lambda: ops.conv(x, pw, out=out, gn_out=True, **kw)
    f0 = lambda: ops.conv(x, pw, out=out, gn_out=False, **kw)
    r1, r0 = [], []
    for _ in range(3):
        r0.append(timed(f0))
        r1.append(timed(f1))
    t1, t0 = sorted(r1)[1], sorted(r0)[1]
    print(f"{name:28s} path {path}: with column sums {t1:9.1f} us, without {t0:9.1f} us, cost {t1 - t0:+8.1f} us "
          f"({(t1 - t0) / t0 * 100:+.1f} %)")
