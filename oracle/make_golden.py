"""Golden-vector generator: imports the READ-ONLY reference at /root/reference
(with the stub packages in oracle/refshim standing in for diffusers 0.32.2 and
ffmpeg-python, and a pre-seeded ``latentsync.utils.util`` -- SURVEY.md Appendix D),
overwrites every parameter with latentsync_amd.weights' deterministic generator
and records inputs/outputs as small .npz fixtures under tests/golden/.

TEST INFRASTRUCTURE ONLY -- run in the build container, never on the GPU box:

    PYTHONDONTWRITEBYTECODE=1 python oracle/make_golden.py [--skip-full]

Only the produced data files are committed, never reference source.
"""
import argparse
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")

sys.path.insert(0, REPO)
from latentsync_amd.weights import randomize_module_  # noqa: E402
from latentsync_amd.config import STAGE2_MODEL, TINY_MODEL, load_model_config  # noqa: E402


def import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(HERE, "refshim"))
    sys.path.insert(1, REF)
    util = types.ModuleType("latentsync.utils.util")
    util.zero_rank_log = lambda logger, msg: None
    sys.modules["latentsync.utils.util"] = util
    import latentsync.models.unet as unet
    import latentsync.models.resnet as resnet
    import latentsync.models.attention as attention
    import latentsync.models.motion_module as motion
    return unet, resnet, attention, motion


def g(seed):
    return torch.Generator().manual_seed(seed)


def randn(shape, seed):
    return torch.randn(shape, generator=g(seed), dtype=torch.float32)


def save(name, **arrays):
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in arrays.items()})
    print("wrote", path, os.path.getsize(path))


@torch.no_grad()
def gen_blocks(resnet, attention, motion):
    torch.manual_seed(0)
    # ResnetBlock3D (resnet.py:104-223), channel change -> conv_shortcut, B=2
    m = resnet.ResnetBlock3D(in_channels=64, out_channels=96, temb_channels=128, groups=32, eps=1e-5,
                             use_inflated_groupnorm=False).eval()
    randomize_module_(m, 11)
    x, temb = randn((2, 64, 4, 8, 8), 1), randn((2, 128), 2)
    save("resnet3d.npz", x=x, temb=temb, out=m(x, temb), seed=11)
    # identity shortcut
    m = resnet.ResnetBlock3D(in_channels=64, out_channels=64, temb_channels=128, groups=32, eps=1e-5,
                             use_inflated_groupnorm=False).eval()
    randomize_module_(m, 12)
    x = randn((1, 64, 4, 8, 8), 3)
    save("resnet3d_id.npz", x=x, temb=temb[:1], out=m(x, temb[:1]), seed=12)
    # Down/Upsample3D
    d = resnet.Downsample3D(64, use_conv=True, out_channels=64, padding=1).eval()
    randomize_module_(d, 13)
    u = resnet.Upsample3D(64, use_conv=True, out_channels=64).eval()
    randomize_module_(u, 14)
    x = randn((1, 64, 4, 8, 8), 4)
    save("samplers.npz", x=x, down=d(x), up=u(x), seed_down=13, seed_up=14)
    # Transformer3DModel with audio cross-attention (attention.py:15-280)
    t = attention.Transformer3DModel(8, 8, in_channels=64, num_layers=1, cross_attention_dim=384,
                                     norm_num_groups=32, add_audio_layer=True).eval()
    randomize_module_(t, 15)
    x, audio = randn((2, 64, 4, 8, 8), 5), randn((8, 50, 384), 6)
    save("transformer3d.npz", x=x, audio=audio, out=t(x, encoder_hidden_states=audio).sample, seed=15)
    # VanillaTemporalModule (motion_module.py:39-313), 16 frames, pos-enc
    mm = motion.VanillaTemporalModule(in_channels=64, num_attention_heads=8, num_transformer_block=1,
                                      attention_block_types=("Temporal_Self", "Temporal_Self"),
                                      temporal_position_encoding=True, temporal_position_encoding_max_len=24,
                                      zero_initialize=True).eval()
    randomize_module_(mm, 16)
    x = randn((1, 64, 16, 4, 4), 7)
    save("motion.npz", x=x, out=mm(x, None, None), seed=16)


@torch.no_grad()
def gen_unet(unet_mod, cfg, name, seed, cases):
    model = unet_mod.UNet3DConditionModel(**cfg).eval()
    randomize_module_(model, seed)
    out = {"seed": seed, "nparams": sum(p.numel() for p in model.parameters())}
    sdict = model.state_dict()
    out["keys"] = np.array(list(sdict.keys()))
    out["shapes"] = np.array([list(v.shape) + [0] * (4 - v.dim()) for v in sdict.values()], dtype=np.int64)
    for i, (B, Fr, H, t, cfg_on) in enumerate(cases):
        sample = randn((B, cfg["in_channels"], Fr, H, H), 100 + i)
        audio = randn((B * Fr, 50, cfg["cross_attention_dim"]), 200 + i)
        if cfg_on:  # CFG batch layout of lipsync_pipeline.py:505-507
            audio[: Fr] = 0
        y = model(sample, t, encoder_hidden_states=audio).sample
        out[f"case{i}_shape"] = np.array([B, Fr, H, t, int(cfg_on)])
        out[f"case{i}_in_sum"] = sample.double().sum().numpy()
        out[f"case{i}_out"] = y
    save(name, **out)


@torch.no_grad()
def gen_whisper():
    sys.modules.setdefault("ffmpeg", types.ModuleType("ffmpeg"))
    from latentsync.whisper.whisper.model import Whisper, ModelDimensions
    from latentsync.whisper.whisper.audio import log_mel_spectrogram, mel_filters
    from latentsync.whisper import audio2feature
    model = Whisper(ModelDimensions(80, 1500, 384, 6, 4, 51865, 448, 384, 6, 4)).eval()
    randomize_module_(model, 21)
    sr = 16000
    tt = np.arange(int(2.5 * sr)) / sr
    rs = np.random.RandomState(1)
    wave = (0.3 * np.sin(2 * np.pi * (220 + 300 * tt) * tt) + 0.05 * rs.randn(tt.size)).astype(np.float32)
    mel = log_mel_spectrogram(wave)
    a2f = object.__new__(audio2feature.Audio2Feature)
    a2f.model, a2f.embedding_dim, a2f.audio_feat_length = model, 384, [2, 2]
    a2f.num_frames, a2f.audio_embeds_cache_dir = 16, None
    res = sys.modules["latentsync.whisper.whisper.transcribe"].transcribe(model, wave, fp16=False)
    feat = []
    for emb in res["segments"]:
        e = emb["encoder_embeddings"].transpose(0, 2, 1, 3).squeeze(0)
        feat.append(e[: int((int(emb["end"]) - int(emb["start"])) / 2)])
    feat = np.concatenate(feat, 0)
    chunks = a2f.feature2chunks(torch.from_numpy(feat), fps=25)
    save("whisper.npz", wave=wave, mel=mel, mel_filters=mel_filters("cpu").numpy(), feature=feat,
         chunks=torch.stack(chunks[:8]), nchunks=len(chunks), seed=21)


def gen_indices():
    from latentsync.whisper import audio2feature
    import latentsync.utils.repeat as rep
    a2f = object.__new__(audio2feature.Audio2Feature)
    a2f.embedding_dim, a2f.audio_feat_length = 1, [2, 2]
    out = {}
    for T in (1, 7, 37, 480):
        feat = torch.arange(T, dtype=torch.float32)[:, None, None].expand(T, 5, 1).contiguous()
        for fps in (25, 30):
            ch = a2f.feature2chunks(feat, fps=fps)
            out[f"T{T}_fps{fps}"] = torch.stack([c[::5, 0] for c in ch]).to(torch.int64)  # (n, 10) indices
    tens = lambda n: [torch.full((2, 3), float(i)) for i in range(n)]
    for n in (1, 15, 16, 17, 242):
        ch, au, dur = rep.pad_whisper_chunks_end(tens(n), (2, 3), torch.zeros(n * 640), 16000, 25)
        out[f"pad_end_{n}"] = np.array([len(ch), au.shape[0], int(round(dur * 1e6))])
        ch, au, dur, k = rep.pad_whisper_chunks(tens(n), (2, 3), torch.zeros(n * 640), 16000, 25)
        out[f"pad_start_{n}"] = np.array([len(ch), au.shape[0], int(round(dur * 1e6)), k, float(ch[-1][0, 0])])
        ch, au, dur = rep.pad_whisper_chunks_to_target(tens(n), (2, 3), torch.zeros(n * 640), 16000, n + 5, 25)
        out[f"pad_target_{n}"] = np.array([len(ch), au.shape[0], int(round(dur * 1e6))])
        out[f"repeat_{n}"] = np.array(rep.repeat_to_length(list(range(n)), 40))
        out[f"trunc_{n}"] = np.array(rep.truncate_to_length(list(range(n)), 10))
    save("indices.npz", **out)


def gen_mask():
    from PIL import Image
    m = np.array(Image.open(os.path.join(REF, "latentsync/utils/mask.png")))
    assert (m[..., 0] == m[..., 1]).all() and (m[..., 0] == m[..., 2]).all()
    save("mask256.npz", bits=np.packbits(m[..., 0] > 127))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-full", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    unet, resnet, attention, motion = import_reference()
    want = lambda k: (not a.only) or k in a.only.split(",")
    ref_cfg = load_model_config(os.path.join(REF, "configs/unet/stage2.yaml"))
    assert ref_cfg == STAGE2_MODEL, "embedded STAGE2_MODEL drifted from configs/unet/stage2.yaml"
    if want("mask"):
        gen_mask()
    if want("indices"):
        gen_indices()
    if want("blocks"):
        gen_blocks(resnet, attention, motion)
    if want("tiny"):
        gen_unet(unet, TINY_MODEL, "unet_tiny.npz", 31,
                 [(1, 16, 32, 951, False), (2, 8, 16, 501, True), (1, 1, 32, 1, False),
                  (1, 16, 64, 951, False), (2, 16, 64, 501, True)])  # configs[4] latent 64^2
    if want("whisper"):
        gen_whisper()
    if want("full") and not a.skip_full:
        gen_unet(unet, STAGE2_MODEL, "unet_full.npz", 41, [(1, 16, 32, 951, False), (1, 1, 32, 1, False),
                  (2, 16, 32, 501, True)])  # CFG batch (configs[2])


if __name__ == "__main__":
    main()
