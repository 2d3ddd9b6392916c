"""Block-level parity on MI355X against golden vectors from the reference's own
ResnetBlock3D / Transformer3DModel / VanillaTemporalModule / samplers
(tests/golden/*.npz), run through the same device-side layer objects the
UNet uses."""
from collections import OrderedDict

import pytest
import torch

from conftest import golden, block_sd, rel_err
from latentsync_amd import ops, schema as S
from latentsync_amd.config import STAGE2_MODEL
from latentsync_amd.unet import _Dev, _Motion, _Resnet, _Transformer

pytestmark = pytest.mark.gpu
TOL = 2e-2


def _shapes(fn, *a):
    sd = OrderedDict()
    fn(sd, "blk", *a)
    return OrderedDict((k[4:], v) for k, v in sd.items())


def to_nhwc(x5):  # (B, C, F, H, W) -> (B*F, H, W, C) bf16 cuda
    B, C, F, H, W = x5.shape
    return x5.permute(0, 2, 3, 4, 1).reshape(B * F, H, W, C).to(torch.bfloat16).cuda().contiguous()


def from_nhwc(y, B):
    n, H, W, C = y.shape
    return y.float().cpu().reshape(B, n // B, H, W, C).permute(0, 4, 1, 2, 3)


@pytest.mark.parametrize("name,cin,cout", [("resnet3d.npz", 64, 96), ("resnet3d_id.npz", 64, 64)])
def test_resnet_block(gpu, name, cin, cout):
    g = golden(name)
    sd = block_sd("blk", _shapes(S._resnet, cin, cout, 128), int(g["seed"]))
    dv = _Dev(sd, torch.device("cuda"))
    r = _Resnet(dv, "blk", cin, cout, 32, 1e-5, 1.0, 0)
    x = torch.from_numpy(g["x"])
    B = x.shape[0]
    w = sd["blk.time_emb_proj.weight"].to(torch.bfloat16).cuda()
    temb = ops.small_linear(torch.from_numpy(g["temb"]).cuda(), w, sd["blk.time_emb_proj.bias"].cuda(), silu_in=True)
    y = r(to_nhwc(x), B, temb)
    e = rel_err(from_nhwc(y, B), g["out"])
    print(name, e)
    assert e < TOL


def test_transformer_block(gpu):
    g = golden("transformer3d.npz")
    sd = block_sd("blk", _shapes(S._transformer, 64, 384, True), int(g["seed"]))
    t = _Transformer(_Dev(sd, torch.device("cuda")), "blk", 64, 8, 32, True)
    x = torch.from_numpy(g["x"])
    audio = torch.from_numpy(g["audio"]).to(torch.bfloat16).cuda().reshape(-1, 384)
    y = t(to_nhwc(x), audio, 50)
    e = rel_err(from_nhwc(y, x.shape[0]), g["out"])
    print("transformer3d", e)
    assert e < TOL


def test_motion_module(gpu):
    g = golden("motion.npz")
    kw = STAGE2_MODEL["motion_module_kwargs"]
    sd = block_sd("blk", _shapes(S._motion, 64, kw), int(g["seed"]))
    m = _Motion(_Dev(sd, torch.device("cuda")), "blk", 64, 8, 32, kw)
    x = torch.from_numpy(g["x"])
    y = m(to_nhwc(x), x.shape[0])
    e = rel_err(from_nhwc(y, x.shape[0]), g["out"])
    print("motion", e)
    assert e < TOL


def test_samplers(gpu):
    g = golden("samplers.npz")
    x = torch.from_numpy(g["x"])
    for key, seed, kw in (("down", "seed_down", dict(stride=2, pad=1)), ("up", "seed_up", dict(upsample=True))):
        shp = OrderedDict([("conv.weight", (64, 64, 3, 3)), ("conv.bias", (64,))])
        sd = block_sd("blk", shp, int(g[seed]))
        pw = _Dev(sd, torch.device("cuda")).packed("blk.conv.weight", "blk.conv.bias")
        y = ops.conv(to_nhwc(x), pw, **kw)
        assert rel_err(from_nhwc(y, 1), g[key]) < 1e-2
