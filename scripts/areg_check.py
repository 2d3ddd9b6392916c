"""A/B correctness: the A-in-registers 1x1 path (tuning key 14) against the
LDS-DMA path on the UNet's 1x1 / 3x3 shapes (bit-identical accumulation order expected)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from latentsync_amd import ops, _lib
from latentsync_amd.packing import pack_weight

lib = _lib.load()
lib.ls_set_tuning(8, 0)  # 3x3 through the tiled GEMM, not the halo conv
torch.manual_seed(0)
bad = 0
for (n, H, cin, c2, cout, ks, ups, res) in [(2, 32, 320, 0, 320, 1, 0, 1), (2, 16, 640, 0, 640, 1, 0, 0),
                                             (2, 8, 1280, 0, 1280, 1, 0, 1), (1, 32, 320, 320, 320, 1, 0, 0),
                                             (2, 16, 640, 0, 640, 3, 0, 0), (1, 16, 640, 640, 640, 3, 0, 1),
                                             (1, 8, 640, 0, 640, 3, 1, 0), (1, 13, 320, 0, 200, 1, 0, 0)]:
    x = torch.randn(n, H, H, cin, device="cuda").to(torch.bfloat16)
    x2 = torch.randn(n, H, H, c2, device="cuda").to(torch.bfloat16) if c2 else None
    w = torch.randn(cout, cin + c2, ks, ks) / ((cin + c2) * ks * ks) ** 0.5
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), torch.randn(cout, device="cuda"), cin + c2, ks, cout)
    Ho = H * 2 if ups else H
    kw = {}
    if x2 is not None:
        kw["x2"] = x2
    if ups:
        kw["upsample"] = True
    if res:
        kw["res"] = torch.randn(n, Ho, Ho, cout, device="cuda").to(torch.bfloat16)
    outs = []
    for rs in (0, 1):
        lib.ls_set_tuning(14, rs)
        outs.append(ops.conv(x, pw, **kw).float())
    torch.cuda.synchronize()
    d = (outs[0] - outs[1]).abs().max().item()
    print(f"n={n} H={H} cin={cin}+{c2} cout={cout} ks={ks} ups={ups} res={res}: max|dma-areg| {d:.3g}", flush=True)
    bad += d > 0
lib.ls_set_tuning(14, 0)
lib.ls_set_tuning(8, 1)
sys.exit(1 if bad else 0)
