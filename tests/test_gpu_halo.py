"""The halo-tile 3x3 conv (conv3x3_halo_kernel, ls_conv_path 3): a 16 x 16 (128-column tiles: 16 x 8) patch of
output pixels per block, its (16 + 2)^2 input pixels loaded once per 64-channel chunk
into LDS and put through the GroupNorm affine + SiLU there (resnet.py:185-213 /
diffusers ResnetBlock2D: conv(silu(GN(x)))), the 9 taps read from that image.  Checked
against fp32 PyTorch (F.conv2d of the activated input) and against the tiled
implicit-GEMM path of the same call (the halo kernel switched off), including the
producer-side GroupNorm column sums, the dual-source concat of the UNet up blocks, the
per-frame row vector (temb), the residual and 5-D GroupNorm samples of F frames."""
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_err
from latentsync_amd import _lib, ops
from latentsync_amd.packing import pack_weight

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(t):
    return t.to(torch.bfloat16).float()


@pytest.mark.parametrize("n,H,W,C1,C2,N,ipp,aff,rowvec,res", [
    (2, 64, 64, 128, 0, 128, 1, True, False, True),      # VAE resnet conv2 (128 ch), residual
    (1, 256, 256, 128, 0, 128, 1, True, False, False),   # VAE 256^2
    (8, 32, 32, 320, 0, 320, 4, True, True, False),      # UNet conv1 at 32^2: 5-D GN over 4 frames, temb row
    (4, 32, 32, 320, 320, 320, 4, True, True, False),    # up-block conv1: cat(h, skip), GN over both
    (4, 16, 16, 640, 0, 640, 2, False, False, True),     # no affine, residual
    (2, 32, 32, 512, 0, 512, 1, True, False, False),     # VAE 512 ch (BN 128, 8 chunks)
    (3, 48, 16, 64, 0, 256, 3, True, False, False),      # one 64-channel chunk, non-square
    # 128-column tiles (16 x 8 form at th8 = 1) with the per-frame row vector AND the residual
    # over a 4-frame GN sample (the TH = 8 epilogue row mapping with both)
    (4, 32, 32, 128, 0, 256, 4, True, True, True),
])
@pytest.mark.parametrize("th8", [1, 0])
def test_halo_conv(gpu, n, H, W, C1, C2, N, ipp, aff, rowvec, res, th8):
    """th8: 128-column tiles (Cin <= 256) on 16 x 8 patches, two blocks per CU (tuning key 16, the
    default) or on the 16 x 16 one-block form; 160-column tiles are 16 x 16 either way."""
    lib = _lib.load()
    if N % 160 == 0 and not th8:
        pytest.skip("160-column tiles have one patch form")
    assert lib.ls_set_tuning(16, th8) == 0
    try:
        _halo_case(lib, n, H, W, C1, C2, N, ipp, aff, rowvec, res)
    finally:
        lib.ls_set_tuning(16, 1)


def _halo_case(lib, n, H, W, C1, C2, N, ipp, aff, rowvec, res):
    g = torch.Generator().manual_seed(n * 1000 + H + C1 + C2 + N)
    Cin = C1 + C2
    x = _bf(torch.randn(n, H, W, C1, generator=g) * 2 + 0.5)
    x2 = _bf(torch.randn(n, H, W, C2, generator=g)) if C2 else None
    w = torch.randn(N, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5
    b = 0.1 * torch.randn(N, generator=g)
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).to(DEV), b.to(DEV), Cin, 3, N)
    S = n // ipp
    scale = (1 + 0.2 * torch.randn(S, Cin, generator=g)).float()
    shift = (0.3 * torch.randn(S, Cin, generator=g)).float()
    tv = torch.randn(n, N, generator=g) if rowvec else None  # one row per frame
    rv = _bf(torch.randn(n, H, W, N, generator=g)) if res else None
    xd = x.to(torch.bfloat16).to(DEV)
    x2d = x2.to(torch.bfloat16).to(DEV) if x2 is not None else None
    kw = dict(x2=x2d)
    if aff:
        kw["aff"] = (scale.to(DEV), shift.to(DEV), ipp, True)
    if rowvec:
        kw["rowvec"] = (tv.to(DEV), H * W, N)
    if res:
        kw["res"] = rv.to(torch.bfloat16).to(DEV)
    # path 3 = the halo kernel takes this call (affine fused, no materialisation)
    assert ops.conv_path(xd, pw, **kw) == 3
    y = ops.conv(xd, pw, gn_out=True, **kw)
    cs_halo = y.gn_cs.clone()
    lib.ls_set_tuning(8, 0)
    try:
        y_ref_path = ops.conv(xd, pw, gn_out=True, aff_materialize=True, **kw)
    finally:
        lib.ls_set_tuning(8, 1)
    # fp32 reference: conv(silu(x * scale + shift)) + bias (+ row vector) (+ residual)
    xin = torch.cat([x, x2], -1) if x2 is not None else x
    if aff:
        sc = scale.repeat_interleave(ipp, 0)[:, None, None, :]
        sh = shift.repeat_interleave(ipp, 0)[:, None, None, :]
        xin = F.silu(xin * sc + sh)
        xin = _bf(xin)  # the halo image holds bf16 activations, as the materialised path
    ref = F.conv2d(xin.permute(0, 3, 1, 2), w, b, padding=1).permute(0, 2, 3, 1)
    if rowvec:
        ref = ref + tv[:, None, None, :]
    if res:
        ref = ref + rv
    yc = y.float().cpu()
    e = rel_err(yc, ref)
    e2 = rel_err(yc, y_ref_path.float().cpu())
    print(f"halo conv {n}x{H}x{W} {C1}+{C2}->{N}: rel vs fp32 {e:.2e}, vs tiled path {e2:.2e}")
    assert e < 1e-2 and e2 < 1e-2
    # GroupNorm column sums of the stored output, per 128-row slot: same per-sample totals
    # as the tiled path's (the slots are numbered by patch, so compare per-sample sums)
    cs_ref = y_ref_path.gn_cs
    per_s = lambda cs: cs.view(S, -1, 2, N).double().sum(1)
    assert torch.allclose(per_s(cs_halo), per_s(cs_ref), rtol=2e-3, atol=1e-2 * H * W * ipp ** 0.5)


def test_halo_conv_path_code(gpu):
    """ls_conv_path reports 3 for the calls the halo kernel takes (so ops.conv passes the
    affine through instead of materialising it) and not for strided / 1x1 / W % 16 convs."""
    lib = _lib.load()
    x = torch.zeros(2, 32, 32, 128, dtype=torch.bfloat16, device=DEV)
    w = torch.zeros(128, 128, 3, 3)
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).to(DEV), torch.zeros(128, device=DEV), 128, 3, 128)
    assert ops.conv_path(x, pw) == 3
    x8 = torch.zeros(2, 8, 8, 128, dtype=torch.bfloat16, device=DEV)
    assert ops.conv_path(x8, pw) != 3
    assert ops.conv_path(x, pw, stride=2, pad=1) != 3


@pytest.mark.parametrize("n,H,W,Cin,N,res", [
    (4, 16, 16, 640, 640, False),     # the UNet's 16x16 -> 32x32 upsampler conv (up_blocks.1)
    (2, 8, 16, 128, 256, True),       # 128-column tiles (16 x 8 patches), residual, non-square
    (2, 32, 32, 256, 256, False),     # a VAE-like upsampler conv
])
def test_halo_conv_upsample(gpu, n, H, W, Cin, N, res):
    """Nearest-x2 upsample + 3x3 conv (Upsample3D, resnet.py:53-71) on the halo kernel (tuning
    key 18): halo pixel (y, x) of the output reads input pixel (y >> 1, x >> 1).  Against fp32
    (F.interpolate nearest + F.conv2d) and the tiled gather path, with the GroupNorm column sums."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(n * 100 + H + Cin + N)
    x = _bf(torch.randn(n, H, W, Cin, generator=g))
    w = torch.randn(N, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5
    b = 0.1 * torch.randn(N, generator=g)
    rv = _bf(torch.randn(n, 2 * H, 2 * W, N, generator=g)) if res else None
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).to(DEV), b.to(DEV), Cin, 3, N)
    xd = x.to(torch.bfloat16).to(DEV)
    kw = dict(upsample=True)
    if res:
        kw["res"] = rv.to(torch.bfloat16).to(DEV)
    assert ops.conv_path(xd, pw, **kw) == 3
    y = ops.conv(xd, pw, gn_out=True, **kw)
    cs = y.gn_cs.clone()
    assert lib.ls_set_tuning(18, 0) == 0
    try:
        assert ops.conv_path(xd, pw, **kw) != 3
        y2 = ops.conv(xd, pw, gn_out=True, **kw)
    finally:
        lib.ls_set_tuning(18, 1)
    up = F.interpolate(x.permute(0, 3, 1, 2), scale_factor=2.0, mode="nearest")
    ref = F.conv2d(up, w, b, padding=1).permute(0, 2, 3, 1)
    if res:
        ref = ref + rv
    e, e2 = rel_err(y.float().cpu(), ref), rel_err(y.float().cpu(), y2.float().cpu())
    print(f"halo upsample conv {n}x{H}x{W} {Cin}->{N}: rel vs fp32 {e:.2e}, vs tiled gather {e2:.2e}")
    assert y.shape == (n, 2 * H, 2 * W, N) and e < 1e-2 and e2 < 1e-2
    tot = lambda c: c.view(n, -1, 2, N).double().sum(1)
    assert torch.allclose(tot(cs), tot(y2.gn_cs), rtol=2e-3, atol=1e-2 * 4 * H * W)


@pytest.mark.parametrize("n,H,W,Cin,N,n_real,res", [
    (2, 256, 256, 128, 8, 3, False),  # the VAE decoder's conv_out: 3 RGB channels padded to 8
    (4, 32, 32, 512, 8, 8, False),    # the encoder's conv_out (2 x 4 latent moments)
    (3, 32, 48, 64, 16, 16, True),    # 16 columns, one chunk, residual, non-square
])
def test_halo_conv_narrow(gpu, n, H, W, Cin, N, n_real, res):
    """The narrow 16-column halo tile (N <= 16, tuning key 19): one channel wave, 16 x 8 patches,
    weight rows past N read as zeros (buffer descriptor bound), with the GroupNorm affine + SiLU
    of conv_norm_out fused (diffusers Decoder / Encoder: conv_out(silu(conv_norm_out(h)))).
    Against fp32 and the tiled 128 x 32 GEMM on the materialised input, with column sums."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(n * 10 + H + Cin + N)
    x = _bf(torch.randn(n, H, W, Cin, generator=g) * 2 + 0.5)
    w = torch.zeros(N, Cin, 3, 3)
    w[:n_real] = torch.randn(n_real, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5
    b = torch.zeros(N)
    b[:n_real] = 0.1 * torch.randn(n_real, generator=g)
    scale = (1 + 0.2 * torch.randn(n, Cin, generator=g)).float()
    shift = (0.3 * torch.randn(n, Cin, generator=g)).float()
    rv = _bf(torch.randn(n, H, W, N, generator=g)) if res else None
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).to(DEV), b.to(DEV), Cin, 3, N)
    xd = x.to(torch.bfloat16).to(DEV)
    kw = dict(aff=(scale.to(DEV), shift.to(DEV), 1, True))
    if res:
        kw["res"] = rv.to(torch.bfloat16).to(DEV)
    assert ops.conv_path(xd, pw, **kw) == 3
    y = ops.conv(xd, pw, gn_out=True, **kw)
    cs = y.gn_cs.clone()
    assert lib.ls_set_tuning(19, 0) == 0
    try:
        assert ops.conv_path(xd, pw, **kw) != 3
        y2 = ops.conv(xd, pw, gn_out=True, aff_materialize=True, **kw)
    finally:
        lib.ls_set_tuning(19, 1)
    xin = _bf(F.silu(x * scale[:, None, None, :] + shift[:, None, None, :]))
    ref = F.conv2d(xin.permute(0, 3, 1, 2), w, b, padding=1).permute(0, 2, 3, 1)
    if res:
        ref = ref + rv
    yc = y.float().cpu()
    e, e2 = rel_err(yc, ref), rel_err(yc, y2.float().cpu())
    print(f"narrow halo conv {n}x{H}x{W} {Cin}->{N} ({n_real} used): rel vs fp32 {e:.2e}, vs tiled {e2:.2e}")
    assert y.shape == (n, H, W, N) and e < 1e-2 and e2 < 1e-2
    if not res and n_real < N:  # the padded columns are exact zeros
        assert yc[..., n_real:].abs().max().item() == 0.0
    tot = lambda c: c.view(n, -1, 2, N).double().sum(1)
    assert torch.allclose(tot(cs), tot(y2.gn_cs), rtol=2e-3, atol=1e-2 * H * W)
