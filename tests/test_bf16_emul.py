"""The bf16-storage emulation of the oracle (oracle/bf16_emul.py), the yardstick of the
served-window per-pixel bound (tests/test_serve_gpu.py): it rounds, it restores torch's
functions afterwards, and on the tiny configuration its distance from the fp32 oracle is of
the size the GPU's is (max 8, p99.9 4-5 levels in the mouth region)."""
import os

import numpy as np
import torch
import torch.nn.functional as F

from latentsync_amd.config import TINY_MODEL
from latentsync_amd.unet import UNet3DConditionModel
from latentsync_amd.vae import AutoencoderKL
from oracle import align_cpu as A
from oracle import ref_cpu as R
from oracle.bf16_emul import bf16_storage, bf16_weights


def test_bf16_storage_rounds_and_restores():
    x = torch.tensor([1.0 + 2 ** -10])
    conv, silu = F.conv2d, F.silu
    with bf16_storage():
        y = F.linear(x[None], torch.ones(1, 1))
        assert y.item() == 1.0  # 1 + 2^-10 is not a bf16 value
    assert F.conv2d is conv and F.silu is silu
    assert bf16_weights({"w": x})["w"].item() == 1.0


def test_tiny_window_bf16_deviation(monkeypatch):
    torch.set_num_threads(8)
    FR, RR, VAE_CH = 8, 64, (32, 64, 64, 64)
    monkeypatch.setitem(R.VAE_CFG, "block_out_channels", VAE_CH)
    unet = UNet3DConditionModel(**TINY_MODEL).init_weights(3)
    vae = AutoencoderKL(block_out_channels=VAE_CH).init_weights(4)
    g = torch.Generator().manual_seed(5)
    faces = (torch.rand((FR, 3, RR, RR), generator=g) * 255).to(torch.uint8)
    import latentsync_amd
    bits = np.load(os.path.join(os.path.dirname(latentsync_amd.__file__), "assets", "fix_mask_256.npz"))["bits"]
    m256 = (np.unpackbits(bits)[: 256 * 256].reshape(256, 256) * 255).astype(np.uint8)
    mask = torch.from_numpy(A.resize_lanczos4_u8(m256, RR, RR).astype(np.float64) / 255.0).float()
    audio = torch.randn((FR, 50, 384), generator=g)
    h = RR // 8
    init = torch.randn((1, 4, 1, h, h), generator=g)
    em, er = torch.randn((FR, 4, h, h), generator=g), torch.randn((FR, 4, h, h), generator=g)
    args = (faces, mask, audio, init, em, er)
    with torch.no_grad():
        ref = R.pipeline_window(unet.state_dict(), dict(unet.config), vae._sd, *args, num_steps=2, guidance_scale=1.5)
        with bf16_storage():
            emu = R.pipeline_window(bf16_weights(unet.state_dict()), dict(unet.config), bf16_weights(vae._sd), *args,
                                    num_steps=2, guidance_scale=1.5)
    u8 = lambda x: ((x / 2 + 0.5).clamp(0, 1) * 255).to(torch.uint8).to(torch.float64)
    d = (u8(ref) - u8(emu)).abs()
    rel = float((emu - ref).norm() / ref.norm())
    print(f"bf16-emulated vs fp32 oracle, tiny window: rel {rel:.4f} max {float(d.max()):.0f} "
          f"p99.9 {float(torch.quantile(d.flatten(), 0.999)):.0f}")
    assert 1e-3 < rel < 3e-2 and d.max() >= 2
