"""Window-level parity: WindowEngine (graph-captured HIP path) against the CPU
oracle's pipeline_window (lipsync_pipeline.py:500-575 restated) on a reduced
configuration (tiny UNet, reduced-width VAE, 64x64 faces) with injected noise,
with and without classifier-free guidance."""
import pytest
import torch

from conftest import rel_err
from latentsync_amd.config import TINY_MODEL
from latentsync_amd.pipeline import WindowEngine, load_fixed_mask
from latentsync_amd.scheduler import DDIMScheduler
from latentsync_amd.unet import UNet3DConditionModel
from latentsync_amd.vae import AutoencoderKL
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
SCHED = dict(beta_end=0.012, beta_schedule="scaled_linear", beta_start=0.00085, clip_sample=False,
             num_train_timesteps=1000, set_alpha_to_one=False, steps_offset=1)


@pytest.mark.parametrize("guidance,graphs", [(1.0, True), (2.0, True), (1.0, False)])
def test_window_matches_oracle(gpu, guidance, graphs, monkeypatch):
    Fr, Rr, steps = 8, 64, 3
    h = Rr // 8
    unet = UNet3DConditionModel(**TINY_MODEL).init_weights(3).to("cuda").eval()
    vae = AutoencoderKL(block_out_channels=(32, 64, 64, 64)).init_weights(4).to("cuda")
    monkeypatch.setitem(R.VAE_CFG, "block_out_channels", (32, 64, 64, 64))
    g = torch.Generator().manual_seed(5)
    faces = (torch.rand((Fr, 3, Rr, Rr), generator=g) * 255).to(torch.uint8)
    mask = load_fixed_mask(Rr)
    audio = torch.randn((Fr, 50, 384), generator=g)
    init = torch.randn((1, 4, 1, h, h), generator=g)
    em, er = torch.randn((Fr, 4, h, h), generator=g), torch.randn((Fr, 4, h, h), generator=g)
    eng = WindowEngine(unet, vae, DDIMScheduler(**SCHED), Fr, Rr, steps, guidance, use_graphs=graphs)
    eng.load(faces.cuda(), mask.cuda(), audio.cuda(), init.cuda(), em.cuda(), er.cuda())
    out = eng.run().cpu()
    out2 = eng.run().cpu()  # replay must be deterministic
    assert torch.equal(out, out2)
    ref = R.pipeline_window(unet.state_dict(), dict(unet.config), vae._sd, faces, mask, audio, init, em, er,
                            num_steps=steps, guidance_scale=guidance)
    e = rel_err(out, ref)
    print("window rel_err", guidance, graphs, e)
    assert e < 3e-2
    # outside the mouth the original pixels are pasted back exactly (up to bf16 of the prep)
    keep = mask.bool()[None, None].expand_as(ref)
    assert (out[keep] - ref[keep]).abs().max() < 1e-2
