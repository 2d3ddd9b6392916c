"""Whisper-tiny audio front end on MI355X (ls_log_mel, the encoder on the
conv/LN/attention kernels, ls_audio_chunks) against the reference-generated
golden vectors (tests/golden/whisper.npz: randomised Whisper-tiny, seed 21,
2.5 s chirp) and, for a two-segment clip, against the oracle restatement.

Tolerances: log-mel max |err| <= 0.02 (bf16 output of values in [-1.5, 1.5]);
encoder features rel-L2 < 3e-2 (bf16 activations over 2 convs + 4 blocks);
the chunk gather is bit-exact against the same bf16 feature rows."""
import numpy as np
import pytest
import torch

from conftest import golden, rel_err
from latentsync_amd.audio import Audio2Feature

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def enc():
    g = golden("whisper.npz")
    return Audio2Feature.random(seed=int(g["seed"]), device="cuda")


def test_log_mel_vs_golden(enc):
    g = golden("whisper.npz")
    mel = enc.log_mel(torch.from_numpy(g["wave"])).float().cpu().T  # (80, T)
    ref = torch.from_numpy(g["mel"])
    assert mel.shape == ref.shape
    err = (mel - ref).abs().max().item()
    print("log-mel max abs err", err)
    assert err <= 0.02


def test_log_mel_padding(enc):
    g = golden("whisper.npz")
    mel = enc.log_mel(torch.from_numpy(g["wave"]), t_pad=3000).float().cpu()
    assert mel.shape == (3000, 80)
    assert torch.count_nonzero(mel[250:]) == 0


def test_features_and_chunks_vs_golden(enc):
    g = golden("whisper.npz")
    feat = enc.audio2feat(g["wave"])
    assert tuple(feat.shape) == g["feature"].shape and feat.dtype == torch.float32
    e = rel_err(feat.cpu(), g["feature"])
    print("whisper feature rel_err", e)
    assert e < 3e-2
    ch = enc.feature2chunks(feat, fps=25)
    assert len(ch) == int(g["nchunks"])
    e2 = rel_err(torch.stack(ch[:8]).cpu(), g["chunks"])
    print("chunks rel_err", e2)
    assert e2 < 3e-2


@pytest.mark.parametrize("T,fps", [(1, 25), (37, 30), (480, 25)])
def test_chunk_gather_bit_exact(enc, T, fps):
    from oracle import ref_cpu as R
    feat = torch.randn((T, 5, 384), generator=torch.Generator().manual_seed(T)).to(torch.bfloat16).float()
    got = enc.chunks_tensor(feat.cuda(), fps).cpu()
    ref = torch.stack(R.feature2chunks(feat, fps=fps))
    assert got.shape == ref.shape
    assert torch.equal(got, ref)
    got16 = enc.chunks_tensor(feat.cuda(), fps, out_f32=False).cpu()
    assert torch.equal(got16.float(), ref)


def test_two_segment_clip_vs_oracle(enc):
    """> 30 s: two encoder segments (transcribe.py seek loop), clip-global mel max."""
    from oracle import ref_cpu as R
    g = golden("whisper.npz")
    n = 16000 * 33
    t = np.arange(n) / 16000.0
    wave = (0.3 * np.sin(2 * np.pi * (200 + 40 * t) * t) * np.exp(-0.02 * t)).astype(np.float32)
    feat = enc.audio2feat(wave).cpu()
    sd = {k: v for k, v in enc.sd.items()}
    with torch.no_grad():
        ref = R.whisper_features(sd, wave, g["mel_filters"])
    assert feat.shape == ref.shape == (1650, 5, 384)
    e = rel_err(feat, ref)
    print("two-segment feature rel_err", e)
    assert e < 3e-2
