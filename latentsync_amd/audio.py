"""Audio2Feature -- drop-in for latentsync/whisper/audio2feature.py:9-135 with the
Whisper-tiny encoder on the HIP path.

  wave (16 kHz fp32) --ls_log_mel--> bf16 mel [n_seg*3000][80] (frame-major,
      zero pad per 30 s segment: transcribe.py's segment loop + pad_or_trim)
  --conv1 (k3, GELU)--> --conv2 (k3 s2, GELU)--> + positional embedding
      -> X[:, 0]                                     (whisper/model.py:143-156)
  4 x ResidualAttentionBlock: row stats -> fused q|k|v GEMM with attn_ln folded
      in -> flash attention (6 heads, d 64, scale d^-1/2 = the reference's d^-1/4
      on q and k) -> out GEMM (+ residual) -> row stats -> MLP GEMM (mlp_ln
      folded, GELU) -> GEMM (+ residual) -> X[:, l]
                                                      (model.py:29-100, 158-171)
  X is [n_seg*1500][5][384] bf16: every layer writes its residual stream straight
  into its slot of the stacked `encoder_embeddings` (the include_embeddings
  output), so the (T50, 5, 384) feature is X[:T50] with no copy: each full
  30 s segment keeps exactly 1500 rows (audio2feature.py:102-115).
  feature2chunks --ls_audio_chunks--> (n_chunks, 50, 384) on device.

Conv1d runs as the 3x3 implicit-GEMM conv on a 1-row image (kernel on the middle
row, packing.pack_weight).  All arithmetic is in libls_hip.so; there is no CPU
path.
"""
import math
import os
import types
import wave

import numpy as np
import torch

from . import _lib, ops
from ._lib import check
from .schema import whisper_encoder_param_shapes
from .weights import fill_state_dict
from .unet import _Dev

SAMPLE_RATE, N_FFT, HOP, N_FRAMES = 16000, 400, 160, 3000
TINY_DIMS = dict(n_mels=80, n_audio_ctx=1500, n_audio_state=384, n_audio_head=6, n_audio_layer=4)


# ----------------------------------------------------------------- host helpers


def mel_filters(sr=SAMPLE_RATE, n_fft=N_FFT, n_mels=80):
    """Slaney-scale, Slaney-normalised triangular filterbank (librosa.filters.mel
    defaults, the published algorithm behind whisper/assets/mel_filters.npz that
    whisper/audio.py:80-90 loads).  float64 math, float32 result (80, 201)."""
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = math.log(6.4) / 27.0

    def hz_to_mel(f):
        f = np.asarray(f, dtype=np.float64)
        m = f / f_sp
        return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, m)

    def mel_to_hz(m):
        m = np.asarray(m, dtype=np.float64)
        f = f_sp * m
        return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f)

    fftfreqs = np.linspace(0, sr / 2, 1 + n_fft // 2)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(0.0), hz_to_mel(sr / 2), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    weights = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    return (weights * enorm[:, None]).astype(np.float32)


def load_wav(path, sr=SAMPLE_RATE):
    """16-bit PCM WAV -> fp32 mono in [-1, 1).  Stands in for whisper's ffmpeg
    load_audio (audio.py:22-50); other containers / resampling need ffmpeg,
    which is outside this build."""
    with wave.open(path, "rb") as f:
        if f.getsampwidth() != 2:
            raise NotImplementedError(f"{path}: only 16-bit PCM WAV is supported (decode with ffmpeg first)")
        if f.getframerate() != sr:
            raise NotImplementedError(f"{path}: sample rate {f.getframerate()} != {sr} (resample with ffmpeg first)")
        ch = f.getnchannels()
        a = np.frombuffer(f.readframes(f.getnframes()), dtype="<i2").astype(np.float32) / 32768.0
    if ch > 1:
        a = a.reshape(-1, ch).mean(1)
    return a


def read_audio(audio_path, audio_sample_rate=SAMPLE_RATE):
    """utils/util.py:103-112 (mono float samples)."""
    if audio_path is None:
        raise ValueError("Audio path is required.")
    return torch.from_numpy(load_wav(audio_path, audio_sample_rate))


def whisper_sinusoids(length, channels, max_timescale=10000):
    """whisper/model.py:48-54."""
    inc = math.log(max_timescale) / (channels // 2 - 1)
    inv = torch.exp(-inc * torch.arange(channels // 2))
    st = torch.arange(length)[:, None] * inv[None, :]
    return torch.cat([torch.sin(st), torch.cos(st)], dim=1)


def num_chunks(T, fps):
    """feature2chunks' loop count (audio2feature.py:85-100): append, then stop once
    int(i * 50 / fps) > T for the i just appended."""
    mult = 50.0 / fps
    i = 0
    while True:
        start = int(i * mult)
        i += 1
        if start > T:
            return i


# ----------------------------------------------------------------- device encoder


class _DeviceWhisper:
    def __init__(self, sd, dims, device):
        self.dims, self.device = dims, device
        dv = _Dev(sd, device)
        self.C, self.heads = dims["n_audio_state"], dims["n_audio_head"]
        self.n_layer = dims["n_audio_layer"]
        self.conv1 = dv.packed("encoder.conv1.weight", "encoder.conv1.bias", ksize=3)
        self.conv2 = dv.packed("encoder.conv2.weight", "encoder.conv2.bias", ksize=3)
        pe = sd.get("encoder.positional_embedding")
        if pe is None:
            pe = whisper_sinusoids(dims["n_audio_ctx"], self.C)
        self.pos = pe.float().to(device).contiguous()
        self.blocks = []
        for i in range(self.n_layer):
            p = f"encoder.blocks.{i}"
            qb, vb = sd[p + ".attn.query.bias"].float(), sd[p + ".attn.value.bias"].float()
            # attn_ln / mlp_ln folded into the q|k|v and mlp.0 GEMMs (ls_conv_desc.ln_rowstats)
            blk = types.SimpleNamespace(
                qkv=dv.packed_ln(torch.cat([sd[p + f".attn.{n}.weight"].float() for n in ("query", "key", "value")]),
                                 torch.cat([qb, torch.zeros_like(qb), vb]),
                                 (sd[p + ".attn_ln.weight"], sd[p + ".attn_ln.bias"])),
                out=dv.packed(p + ".attn.out.weight", p + ".attn.out.bias"),
                mlp1=dv.packed_ln(sd[p + ".mlp.0.weight"], sd[p + ".mlp.0.bias"],
                                  (sd[p + ".mlp_ln.weight"], sd[p + ".mlp_ln.bias"])),
                mlp2=dv.packed(p + ".mlp.2.weight", p + ".mlp.2.bias"))
            self.blocks.append(blk)

    def encode(self, mel):
        """mel bf16 (n_seg, 1, 3000, 80) -> X bf16 (n_seg * 1500, n_layer + 1, C)."""
        n_seg = mel.shape[0]
        C, L = self.C, self.n_layer + 1
        ctx = self.dims["n_audio_ctx"]
        rows = n_seg * ctx
        h1 = ops.conv(mel, self.conv1, act=ops.ACT_GELU)                             # (n, 1, 3000, C)
        h2 = ops.conv(h1, self.conv2, stride=2, act=ops.ACT_GELU)                   # (n, 1, 1500, C)
        X = torch.empty((rows, L, C), dtype=torch.bfloat16, device=mel.device)
        ops.add_rows(h2.view(rows, C), self.pos, out=X[:, 0])
        d = C // self.heads
        o = torch.empty((rows, C), dtype=torch.bfloat16, device=mel.device)
        for li, b in enumerate(self.blocks):
            x = X[:, li]
            y = X[:, li + 1]
            qkv = ops.linear(x, b.qkv, ln_stats=ops.row_stats(x))
            qs = (ctx * 3 * C, 0, 3 * C, d)
            ops.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=n_seg, z2=1, heads=self.heads, nq=ctx, nk=ctx,
                          head_dim=d, qs=qs, ks=qs, vs=qs, os_=(ctx * C, 0, C, d))
            ops.linear(o, b.out, res=x, out=y)
            m = ops.linear(y, b.mlp1, act=ops.ACT_GELU, ln_stats=ops.row_stats(y))
            ops.linear(m, b.mlp2, res=y, out=y)
        return X


# ----------------------------------------------------------------- drop-in class


class Audio2Feature:
    """audio2feature.py:9-22 constructor; `audio2feat`, `feature2chunks`,
    `get_sliced_feature` keep the reference's signatures and semantics."""

    def __init__(self, model_path="checkpoints/whisper/tiny.pt", device=None, audio_embeds_cache_dir=None,
                 num_frames=16, audio_feat_length=(2, 2), state_dict=None, dims=None):
        if state_dict is None:
            if not model_path or not os.path.isfile(model_path):
                raise RuntimeError(f"Model {model_path} not found")  # whisper/__init__.py:109
            ck = torch.load(model_path, map_location="cpu", weights_only=True)
            dims = dict(ck["dims"])
            state_dict = {k: v for k, v in ck["model_state_dict"].items() if k.startswith("encoder.")}
        self.dims = dict(TINY_DIMS, **(dims or {}))
        self.model = types.SimpleNamespace(dims=types.SimpleNamespace(**self.dims))
        self.sd = state_dict
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.audio_embeds_cache_dir = audio_embeds_cache_dir
        self.num_frames = num_frames
        self.embedding_dim = self.dims["n_audio_state"]
        self.audio_feat_length = list(audio_feat_length)
        self._dev = None
        self._filters = None
        self._last = None  # (fp32 feature returned, bf16 stacked rows it views)

    @classmethod
    def random(cls, seed=0, device=None, **kw):
        """Whisper-tiny encoder with the repo's deterministic per-key weights
        (the parity fixtures' generator, tests/golden/whisper.npz)."""
        sd = fill_state_dict(whisper_encoder_param_shapes(), seed)
        sd["encoder.positional_embedding"] = whisper_sinusoids(1500, 384)
        return cls(model_path=None, device=device, state_dict=sd, **kw)

    def to(self, device):
        self.device = torch.device(device)
        self._dev = None
        return self

    def _require(self):
        _lib.load()
        if self.device.type != "cuda":
            raise RuntimeError("Audio2Feature runs on the HIP device; move it with .to('cuda')")
        if self._dev is None:
            self._dev = _DeviceWhisper(self.sd, self.dims, self.device)
            self._filters = torch.from_numpy(mel_filters(n_mels=self.dims["n_mels"])).to(self.device)
        return self._dev

    # -- mel + encoder --------------------------------------------------
    def log_mel(self, audio, t_pad=None):
        """whisper/audio.py:92-125 on device -> bf16 (t_pad, 80) frame-major."""
        self._require()
        a = torch.as_tensor(audio, dtype=torch.float32).to(self.device).contiguous()
        n = a.numel()
        T = n // HOP
        t_pad = t_pad or T
        nm = self.dims["n_mels"]
        lib = _lib.load()
        ws = torch.empty(lib.ls_log_mel_workspace_bytes(n, nm), dtype=torch.uint8, device=self.device)
        out = torch.empty((t_pad, nm), dtype=torch.bfloat16, device=self.device)
        check(lib.ls_log_mel(a.data_ptr(), n, self._filters.data_ptr(), nm, t_pad, out.data_ptr(), ws.data_ptr(),
                             ws.numel(), ops._stream()), "ls_log_mel")
        return out

    def encode_stacked(self, audio):
        """wave -> (X bf16 (n_seg*1500, 5, 384), T50): transcribe.py:85-128 segment
        loop batched into one encoder pass over all 30 s segments."""
        dev = self._require()
        n = torch.as_tensor(audio).numel()
        T = n // HOP
        n_seg = max(1, math.ceil(T / N_FRAMES))
        mel = self.log_mel(audio, t_pad=n_seg * N_FRAMES)
        X = dev.encode(mel.view(n_seg, 1, N_FRAMES, -1))
        T50 = sum(int((min(s + N_FRAMES, T) - s) / 2) for s in range(0, T, N_FRAMES))
        return X, T50

    def _audio2feat(self, audio):
        if isinstance(audio, str):
            audio = load_wav(audio)
        X, T50 = self.encode_stacked(audio)
        feat = X[:T50].float()
        self._last = (feat, X[:T50])
        return feat

    def audio2feat(self, audio_path):
        """audio2feature.py:117-135 (including the optional embeds cache)."""
        if not self.audio_embeds_cache_dir:
            return self._audio2feat(audio_path)
        path = os.path.join(self.audio_embeds_cache_dir, os.path.basename(audio_path) + ".pt")
        if os.path.isfile(path):
            try:
                return torch.load(path, map_location=self.device, weights_only=True)
            except Exception as e:  # corrupt cache entry: recompute (as the reference does)
                print(f"{type(e).__name__} - {e} - {path}")
                os.remove(path)
        feat = self._audio2feat(audio_path)
        torch.save(feat.cpu(), path)
        return feat

    # -- chunking ---------------------------------------------------------
    def chunks_tensor(self, feature_array, fps, out_f32=True):
        """feature2chunks as one (n_chunks, 50, 384) device tensor."""
        self._require()
        if self._last is not None and feature_array is self._last[0]:
            fb = self._last[1]
        else:
            fb = torch.as_tensor(feature_array).to(self.device, torch.bfloat16).contiguous()
        T, layers, C = fb.shape
        nc = num_chunks(T, fps)
        fl, fr = self.audio_feat_length
        rows = (fl + fr + 1) * 2 * layers
        out = torch.empty((nc, rows, C), dtype=torch.float32 if out_f32 else torch.bfloat16, device=self.device)
        lib = _lib.load()
        check(lib.ls_audio_chunks(fb.data_ptr(), fb.stride(0), T, layers, C, nc, float(fps), fl, fr, out.data_ptr(),
                                  int(out_f32), ops._stream()), "ls_audio_chunks")
        return out

    def feature2chunks(self, feature_array, fps):
        """audio2feature.py:85-100 -> list of (50, 384) chunks."""
        return list(self.chunks_tensor(feature_array, fps).unbind(0))

    def get_sliced_feature(self, feature_array, vid_idx, fps=25):
        """audio2feature.py:24-49 -> ((50, 384), idx list)."""
        length = len(feature_array)
        center = int(vid_idx * 50 / fps)
        left = center - self.audio_feat_length[0] * 2
        right = center + (self.audio_feat_length[1] + 1) * 2
        idx = [min(length - 1, max(0, i)) for i in range(left, right)]
        fa = torch.as_tensor(feature_array)
        return fa[idx].reshape(-1, self.embedding_dim), idx
