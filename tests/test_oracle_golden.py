"""Pins the CPU oracle (oracle/ref_cpu.py) against golden vectors produced by
importing the reference itself (oracle/make_golden.py)."""
from collections import OrderedDict

import numpy as np
import pytest
import torch

from conftest import golden, block_sd, rel_err
from oracle import ref_cpu as R
from latentsync_amd import schema as S
from latentsync_amd.config import STAGE2_MODEL, TINY_MODEL
from latentsync_amd.weights import fill_state_dict

torch.set_num_threads(8)


def _shapes(fn, *a):
    sd = OrderedDict()
    fn(sd, "blk", *a)
    return OrderedDict((k[4:], v) for k, v in sd.items())


def test_resnet3d():
    for name, cin, cout in (("resnet3d.npz", 64, 96), ("resnet3d_id.npz", 64, 64)):
        g = golden(name)
        sd = block_sd("blk", _shapes(S._resnet, cin, cout, 128), int(g["seed"]))
        y = R.resnet_block(torch.from_numpy(g["x"]), torch.from_numpy(g["temb"]), sd, "blk", 32, 1e-5)
        assert rel_err(y, g["out"]) < 1e-5


def test_samplers():
    g = golden("samplers.npz")
    x = torch.from_numpy(g["x"])
    sd = block_sd("blk", OrderedDict([("conv.weight", (64, 64, 3, 3)), ("conv.bias", (64,))]), int(g["seed_down"]))
    assert rel_err(R._inflated_conv(x, sd, "blk.conv", stride=2), g["down"]) < 1e-5
    sd = block_sd("blk", OrderedDict([("conv.weight", (64, 64, 3, 3)), ("conv.bias", (64,))]), int(g["seed_up"]))
    assert rel_err(R._inflated_conv(R.upsample_nearest(x), sd, "blk.conv"), g["up"]) < 1e-5


def test_transformer3d():
    g = golden("transformer3d.npz")
    sd = block_sd("blk", _shapes(S._transformer, 64, 384, True), int(g["seed"]))
    y = R.transformer3d(torch.from_numpy(g["x"]), torch.from_numpy(g["audio"]), sd, "blk", 8, 32)
    assert rel_err(y, g["out"]) < 1e-5


def test_motion_module():
    g = golden("motion.npz")
    kw = STAGE2_MODEL["motion_module_kwargs"]
    sd = block_sd("blk", _shapes(S._motion, 64, kw), int(g["seed"]))
    y = R.motion_module(torch.from_numpy(g["x"]), sd, "blk", 8, 32)
    assert rel_err(y, g["out"]) < 1e-5


def _unet_cases(g):
    i = 0
    while f"case{i}_shape" in g:
        B, Fr, H, t, cfg_on = (int(v) for v in g[f"case{i}_shape"])
        yield i, B, Fr, H, t, bool(cfg_on)
        i += 1


def _check_schema(cfg, g):
    shapes = S.unet_param_shapes(cfg)
    ref = {k: tuple(int(d) for d in s if d) for k, s in zip(g["keys"].tolist(), g["shapes"])}
    assert set(shapes) == set(ref)
    for k, s in shapes.items():
        assert tuple(s) == ref[k], k
    return shapes


def _run_unet_golden(cfg, name, tol):
    g = golden(name)
    shapes = _check_schema(cfg, g)
    sd = fill_state_dict(shapes, int(g["seed"]))
    for i, B, Fr, H, t, cfg_on in _unet_cases(g):
        gen = torch.Generator().manual_seed(100 + i)
        sample = torch.randn((B, cfg["in_channels"], Fr, H, H), generator=gen)
        assert abs(float(sample.double().sum()) - float(g[f"case{i}_in_sum"])) < 1e-6
        audio = torch.randn((B * Fr, 50, cfg["cross_attention_dim"]), generator=torch.Generator().manual_seed(200 + i))
        if cfg_on:
            audio[:Fr] = 0
        with torch.no_grad():
            y = R.unet_forward(sd, cfg, sample, t, audio)
        assert rel_err(y, g[f"case{i}_out"]) < tol, (name, i)


def test_unet_tiny():
    _run_unet_golden(TINY_MODEL, "unet_tiny.npz", 1e-5)


@pytest.mark.slow
def test_unet_full():
    _run_unet_golden(STAGE2_MODEL, "unet_full.npz", 1e-5)


def test_unet_full_schema():
    g = golden("unet_full.npz")
    shapes = _check_schema(STAGE2_MODEL, g)
    assert sum(int(np.prod(s)) for k, s in shapes.items() if not k.endswith(".pe")) == int(g["nparams"])


def test_feature2chunks_indices():
    g = golden("indices.npz")
    for T in (1, 7, 37, 480):
        for fps in (25, 30):
            feat = torch.arange(T, dtype=torch.float32)[:, None, None].expand(T, 5, 1)
            ch = R.feature2chunks(feat, fps=fps)
            got = torch.stack([c[::5, 0] for c in ch]).to(torch.int64).numpy()
            np.testing.assert_array_equal(got, g[f"T{T}_fps{fps}"])


def test_whisper_features():
    g = golden("whisper.npz")
    sd = fill_state_dict(S.whisper_encoder_param_shapes(), int(g["seed"]))
    sd["encoder.positional_embedding"] = R.whisper_sinusoids(1500, 384)
    mel = R.log_mel_spectrogram(g["wave"], g["mel_filters"])
    assert rel_err(mel, g["mel"]) < 1e-6
    with torch.no_grad():
        feat = R.whisper_features(sd, g["wave"], g["mel_filters"])
    assert feat.shape == g["feature"].shape
    assert rel_err(feat, g["feature"]) < 1e-5
    ch = R.feature2chunks(feat, fps=25)
    assert len(ch) == int(g["nchunks"])
    assert rel_err(torch.stack(ch[:8]), g["chunks"]) < 1e-5


def test_ddim_known_answers():
    """SURVEY.md §8(a) a7 known answers (restated diffusers DDIMScheduler)."""
    ac = R.ddim_alphas_cumprod()
    bits = lambda i: int(np.float32(ac[i].item()).view(np.uint32))
    assert bits(0) == 0x3F7FC84B and bits(1) == 0x3F7F9054 and bits(51) == 0x3F73558C
    assert bits(951) == 0x3C059C8B and bits(981) == 0x3BBD405F
    assert R.ddim_timesteps(20).tolist() == list(range(951, 0, -50))
    assert R.ddim_timesteps(50).tolist() == list(range(981, 0, -20))
    assert R.ddim_timesteps(1).tolist() == [1]
