"""A/B correctness: the halo conv's read-pixel piece enumeration (tuning key 12) against the
padded-image one on GroupNorm-affine 3x3 convs (bit-identical outputs expected)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from latentsync_amd import ops, _lib
from latentsync_amd.packing import pack_weight

lib = _lib.load()
torch.manual_seed(0)
bad = 0
for (n, H, W, cin, c2, cout, res) in [(2, 32, 32, 320, 0, 320, 1), (2, 16, 16, 640, 0, 640, 0), (1, 32, 32, 320, 320, 320, 1),
                                      (2, 64, 64, 128, 0, 128, 0), (1, 48, 32, 256, 0, 256, 1)]:
    x = torch.randn(n, H, W, cin, device="cuda").to(torch.bfloat16)
    x2 = torch.randn(n, H, W, c2, device="cuda").to(torch.bfloat16) if c2 else None
    C = cin + c2
    w = torch.randn(cout, C, 3, 3) / (C * 9) ** 0.5
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), torch.randn(cout, device="cuda"), C, 3, cout)
    kw = dict(aff=(torch.rand(n, C, device="cuda") + 0.5, torch.randn(n, C, device="cuda") * 0.1, 1, True),
              aff_materialize=True)
    if x2 is not None:
        kw["x2"] = x2
    if res:
        kw["res"] = torch.randn(n, H, W, cout, device="cuda").to(torch.bfloat16)
    path = ops.conv_path(x, pw, **kw)
    outs = []
    for rp in (0, 1):
        lib.ls_set_tuning(12, rp)
        outs.append(ops.conv(x, pw, **kw).float())
    torch.cuda.synchronize()
    d = (outs[0] - outs[1]).abs().max().item()
    print(f"n={n} {H}x{W} cin={cin}+{c2} cout={cout} res={res} path={path}: max|pad-rp| {d:.3g}", flush=True)
    bad += d > 0 or path != 3
lib.ls_set_tuning(12, 0)
sys.exit(1 if bad else 0)
