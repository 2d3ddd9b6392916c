"""A/B correctness: the persistent halo conv grid (tuning key 13: one block per CU walking
its patches, chunk pipeline across patch boundaries) against one block per patch, on
GroupNorm-affine 3x3 convs with BN 128 (bit-identical outputs and column sums expected)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from latentsync_amd import ops, _lib
from latentsync_amd.packing import pack_weight

lib = _lib.load()
torch.manual_seed(0)
bad = 0
# (n, H, W, cin, c2, cout, res, gn_out): odd chunk counts (192 = 3 chunks), concat, several
# patches per block (n * H * W / 256 patches over ~256 blocks) and fewer patches than CUs
for (n, H, W, cin, c2, cout, res, gno) in [(8, 64, 64, 128, 0, 128, 1, 1), (4, 128, 128, 128, 0, 256, 0, 0),
                                           (2, 32, 48, 192, 0, 128, 1, 0), (3, 64, 32, 128, 128, 256, 1, 1),
                                           (1, 16, 16, 128, 0, 128, 0, 0), (64, 32, 32, 512, 0, 512, 1, 1)]:
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
    if gno:
        kw["gn_out"] = True
    path = ops.conv_path(x, pw, **kw)
    outs, css = [], []
    for pt in (0, 1):
        lib.ls_set_tuning(13, pt)
        y = ops.conv(x, pw, **kw)
        outs.append(y.float())
        css.append(getattr(y, "gn_cs", None))
    torch.cuda.synchronize()
    d = (outs[0] - outs[1]).abs().max().item()
    dc = (css[0] - css[1]).abs().max().item() if css[0] is not None and css[1] is not None else 0.0
    print(f"n={n} {H}x{W} cin={cin}+{c2} cout={cout} res={res} gn_out={gno} path={path}: max|pp-pt| {d:.3g} colsum {dc:.3g}",
          flush=True)
    bad += d > 0 or dc > 0 or path != 3
lib.ls_set_tuning(13, 1)
sys.exit(1 if bad else 0)
