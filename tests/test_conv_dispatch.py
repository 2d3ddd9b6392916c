"""Host-side dispatch of ls_conv2d (ls_conv_path, no launch, runs without a GPU): which kernel
family takes the round-6 shapes.  3 = the halo-tile 3x3 conv (GroupNorm affine + SiLU fused),
2 = the register-staged GEMM (the caller materialises the affine first)."""
import torch

from latentsync_amd import ops
from latentsync_amd.packing import pack_weight


def _pw(n_real, cin, ks=3, n_pad=None):
    w = torch.zeros(n_real, cin, ks, ks)
    n = n_pad or n_real
    return ops.Packed(pack_weight(w, n_pad=n_pad).to(torch.bfloat16), torch.zeros(n), cin, ks, n)


def _aff(samples, cin, ipp=1):
    return (torch.ones(samples, cin), torch.zeros(samples, cin), ipp, True)


def test_vae_conv_out_takes_the_narrow_halo_tile():
    # decoder conv_out: conv_norm_out + SiLU + 3x3 128 -> 3 (padded to 8) at 256^2 (vae.py)
    x = torch.zeros(2, 256, 256, 128, dtype=torch.bfloat16)
    assert ops.conv_path(x, _pw(3, 128, n_pad=8), aff=_aff(2, 128)) == 3
    # 4 padded columns cannot store 16-B rows: the register-staged GEMM (affine materialised)
    assert ops.conv_path(x, _pw(3, 128, n_pad=4), aff=_aff(2, 128)) == 2
    # encoder conv_out: 512 -> 8 moments at 32^2
    xe = torch.zeros(2, 32, 32, 512, dtype=torch.bfloat16)
    assert ops.conv_path(xe, _pw(8, 512), aff=_aff(2, 512)) == 3


def test_unet_conv_out_takes_the_narrow_halo_tile():
    # conv_norm_out over 16-frame samples + SiLU + 3x3 320 -> 4 (padded to 8) at 32^2 (unet.py)
    x = torch.zeros(32, 32, 32, 320, dtype=torch.bfloat16)
    assert ops.conv_path(x, _pw(4, 320, n_pad=8), aff=_aff(2, 320, ipp=16)) == 3


def test_upsample_convs_take_the_halo_kernel():
    xu = torch.zeros(2, 16, 16, 640, dtype=torch.bfloat16)
    assert ops.conv_path(xu, _pw(640, 640), upsample=True) == 3           # UNet 16^2 -> 32^2
    xv = torch.zeros(2, 32, 32, 512, dtype=torch.bfloat16)
    assert ops.conv_path(xv, _pw(512, 512), upsample=True) == 3           # VAE decoder 32^2 -> 64^2 (BN 128)
    xw = torch.zeros(2, 128, 128, 256, dtype=torch.bfloat16)
    assert ops.conv_path(xw, _pw(256, 256), upsample=True) == 3           # VAE decoder 128^2 -> 256^2
    # an upsample conv with an input affine stays on the tiled gather (the halo form has none)
    assert ops.conv_path(xw, _pw(256, 256), upsample=True, aff=_aff(2, 256)) != 3
