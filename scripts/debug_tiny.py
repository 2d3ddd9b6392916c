"""Debug: per-block GPU vs oracle at tiny widths (C=32, d=4) and concat resnets."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from collections import OrderedDict
import torch
from conftest import block_sd, rel_err
from oracle import ref_cpu as R
from latentsync_amd import ops, schema as S
from latentsync_amd.config import STAGE2_MODEL
from latentsync_amd.unet import _Dev, _Motion, _Resnet, _Transformer

def shp(fn, *a):
    sd = OrderedDict(); fn(sd, "blk", *a)
    return OrderedDict((k[4:], v) for k, v in sd.items())
def nh(x5):
    B, C, F, H, W = x5.shape
    return x5.permute(0, 2, 3, 4, 1).reshape(B * F, H, W, C).to(torch.bfloat16).cuda().contiguous()
def fr(y, B):
    n, H, W, C = y.shape
    return y.float().cpu().reshape(B, n // B, H, W, C).permute(0, 4, 1, 2, 3)
g = torch.Generator().manual_seed(0)
dev = torch.device("cuda")
for (c1, c2, cout, F, H) in [(32, 0, 32, 16, 32), (64, 32, 32, 16, 32), (64, 64, 64, 16, 8), (32, 32, 32, 1, 32)]:
    sd = block_sd("blk", shp(S._resnet, c1 + c2, cout, 128), 5)
    x = torch.randn(1, c1 + c2, F, H, H, generator=g)
    te = torch.randn(1, 128, generator=g)
    ref = R.resnet_block(x, te, sd, "blk", 32, 1e-5)
    r = _Resnet(_Dev(sd, dev), "blk", c1 + c2, cout, 32, 1e-5, 1.0, 0)
    temb = ops.small_linear(te.cuda(), sd["blk.time_emb_proj.weight"].to(torch.bfloat16).cuda(), sd["blk.time_emb_proj.bias"].cuda(), silu_in=True)
    xa = nh(x[:, :c1]); xb = nh(x[:, c1:]) if c2 else None
    y = r(xa, 1, temb, x2=xb)
    print("resnet", c1, c2, cout, F, H, rel_err(fr(y, 1), ref))
for C, F, H in [(32, 16, 32), (64, 16, 16), (32, 1, 32)]:
    sd = block_sd("blk", shp(S._transformer, C, 384, True), 6)
    x = torch.randn(1, C, F, H, H, generator=g); au = torch.randn(F, 50, 384, generator=g)
    ref = R.transformer3d(x, au, sd, "blk", 8, 32)
    t = _Transformer(_Dev(sd, dev), "blk", C, 8, 32, True)
    y = t(nh(x), au.to(torch.bfloat16).cuda().reshape(-1, 384), 50)
    print("transformer", C, F, H, rel_err(fr(y, 1), ref))
    kw = STAGE2_MODEL["motion_module_kwargs"]
    sd = block_sd("blk", shp(S._motion, C, kw), 7)
    ref = R.motion_module(x, sd, "blk", 8, 32)
    m = _Motion(_Dev(sd, dev), "blk", C, 8, 32, kw)
    y = m(nh(x), 1)
    print("motion", C, F, H, rel_err(fr(y, 1), ref))
