"""Host-side pieces of the audio front end (no GPU): the mel filterbank
restatement against the reference's own asset values (tests/golden/whisper.npz
`mel_filters`, written from whisper/assets/mel_filters.npz), the feature2chunks
loop count against the reference's index vectors, and WAV reading."""
import wave

import numpy as np
import torch

from latentsync_amd.audio import Audio2Feature, load_wav, mel_filters, num_chunks, read_audio
from conftest import golden


def test_mel_filters_match_reference_asset():
    ref = golden("whisper.npz")["mel_filters"]
    got = mel_filters()
    assert got.shape == ref.shape == (80, 201)
    assert np.abs(got - ref).max() < 1e-7  # float64 math, float32 result: ULP-level agreement


def test_num_chunks_matches_reference_loop():
    g = golden("indices.npz")
    for T in (1, 7, 37, 480):
        for fps in (25, 30):
            assert num_chunks(T, fps) == g[f"T{T}_fps{fps}"].shape[0], (T, fps)
    assert num_chunks(125, 25) == int(golden("whisper.npz")["nchunks"])


def test_get_sliced_feature_indices():
    g = golden("indices.npz")
    enc = Audio2Feature.__new__(Audio2Feature)
    enc.audio_feat_length, enc.embedding_dim = [2, 2], 384
    feat = torch.arange(37, dtype=torch.float32)[:, None, None].expand(37, 5, 384)
    for i, row in enumerate(g["T37_fps30"]):
        f, idx = enc.get_sliced_feature(feat, i, fps=30)
        assert idx == row.tolist()
        assert f.shape == (50, 384) and torch.equal(f[::5, 0], torch.tensor(row, dtype=torch.float32))


def test_read_wav(tmp_path):
    x = (np.sin(np.arange(1600) * 0.05) * 12000).astype("<i2")
    p = str(tmp_path / "a.wav")
    with wave.open(p, "wb") as f:
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(16000)
        f.writeframes(x.tobytes())
    a = load_wav(p)
    assert a.dtype == np.float32 and np.array_equal(a, x.astype(np.float32) / 32768.0)
    assert torch.equal(read_audio(p), torch.from_numpy(a))
