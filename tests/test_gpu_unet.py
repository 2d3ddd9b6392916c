"""UNet3DConditionModel on MI355X (HIP C-ABI path) against the golden vectors
produced by the reference itself (tests/golden/unet_*.npz).

Tolerance: relative L2 error of the (B, 4, F, h, w) noise prediction.  The
HIP path runs bf16 activations / bf16 weights with fp32 accumulation (the
reference runs fp16 on CUDA, scripts/inference.py:33-34); the oracle is fp32."""
import pytest
import torch

from conftest import golden, rel_err
from latentsync_amd.config import STAGE2_MODEL, TINY_MODEL
from latentsync_amd.unet import UNet3DConditionModel

pytestmark = pytest.mark.gpu
TOL = 3e-2


def _cases(g):
    i = 0
    while f"case{i}_shape" in g:
        B, Fr, H, t, cfg_on = (int(v) for v in g[f"case{i}_shape"])
        yield i, B, Fr, H, t, bool(cfg_on)
        i += 1


def _run(cfg, name):
    g = golden(name)
    unet = UNet3DConditionModel(**cfg).init_weights(int(g["seed"])).to("cuda").eval()
    errs = []
    for i, B, Fr, H, t, cfg_on in _cases(g):
        sample = torch.randn((B, cfg["in_channels"], Fr, H, H), generator=torch.Generator().manual_seed(100 + i))
        audio = torch.randn((B * Fr, 50, cfg["cross_attention_dim"]),
                            generator=torch.Generator().manual_seed(200 + i))
        if cfg_on:
            audio[:Fr] = 0
        with torch.no_grad():
            out = unet(sample.cuda(), torch.tensor(t), encoder_hidden_states=audio.cuda()).sample
        assert out.shape == (B, cfg["out_channels"], Fr, H, H)
        e = rel_err(out.float().cpu(), g[f"case{i}_out"])
        errs.append(e)
        print(name, i, "rel_err", e)
    assert max(errs) < TOL, errs


def test_unet_tiny_matches_reference(gpu):
    _run(TINY_MODEL, "unet_tiny.npz")


def test_unet_full_matches_reference(gpu):
    _run(STAGE2_MODEL, "unet_full.npz")
