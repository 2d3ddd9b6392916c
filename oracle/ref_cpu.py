"""CPU oracle: a plain PyTorch-fp32 restatement of the reference's inference
denoising hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline -- never as the thing measured or shipped.  The
product path (``latentsync_amd``) runs exclusively on the HIP C-ABI library.

Every function is written from the reference's behaviour, citing the file:line it
follows (paths relative to the reference root).  Pinning:
  * UNet3DConditionModel and all its blocks, feature2chunks / get_sliced_feature,
    the repeat.py padding helpers and the Whisper AudioEncoder / log-mel are
    pinned against golden vectors produced by importing the reference itself
    (oracle/make_golden.py -> tests/golden/*.npz, tests/test_oracle_golden.py).
  * diffusers 0.32.2 pieces (AutoencoderKL, DDIMScheduler) are not in the
    reference tree and diffusers is not installed: they are restated from the
    published algorithm -- "parity unpinned", except the
    DDIM integer timesteps and alpha-bar known answers of SURVEY.md §8(a) a7.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

# --------------------------------------------------------------------------
# small helpers
# --------------------------------------------------------------------------


def _lin(x, sd, p, bias=True):
    w = sd[p + ".weight"]
    b = sd.get(p + ".bias") if bias else None
    return F.linear(x, w, b)


def _conv(x4, sd, p, stride=1, padding=1):
    return F.conv2d(x4, sd[p + ".weight"], sd.get(p + ".bias"), stride=stride, padding=padding)


def _fold(x5):  # "b c f h w -> (b f) c h w"
    b, c, f, h, w = x5.shape
    return x5.permute(0, 2, 1, 3, 4).reshape(b * f, c, h, w), f


def _unfold(x4, f):  # "(b f) c h w -> b c f h w"
    bf, c, h, w = x4.shape
    return x4.reshape(bf // f, f, c, h, w).permute(0, 2, 1, 3, 4)


def _inflated_conv(x5, sd, p, stride=1, padding=1):
    """InflatedConv3d (latentsync/models/resnet.py:10-18): frames folded into batch."""
    x4, f = _fold(x5)
    return _unfold(_conv(x4, sd, p, stride, padding), f)


def _ln(x, sd, p, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


# --------------------------------------------------------------------------
# diffusers embeddings / feed-forward (restated)
# --------------------------------------------------------------------------


def timestep_embedding(timesteps, dim, flip_sin_to_cos=True, shift=0, max_period=10000):
    """diffusers get_timestep_embedding (called via Timesteps, unet.py:95,376)."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(0, half, dtype=torch.float32) / (half - shift)
    emb = timesteps[:, None].float() * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


def feed_forward(x, sd, p):
    """diffusers FeedForward(GEGLU): attention.py:171, motion_module.py:200."""
    h = _lin(x, sd, p + ".net.0.proj")
    a, g = h.chunk(2, dim=-1)
    return _lin(a * F.gelu(g), sd, p + ".net.2")


def attention(x, sd, p, heads, context=None):
    """latentsync/models/attention.py:250-280 (Attention.forward, SDPA no mask)."""
    ctx = x if context is None else context
    q = _lin(x, sd, p + ".to_q", bias=False)
    k = _lin(ctx, sd, p + ".to_k", bias=False)
    v = _lin(ctx, sd, p + ".to_v", bias=False)

    def split(t):
        b, n, c = t.shape
        return t.reshape(b, n, heads, c // heads).permute(0, 2, 1, 3)

    o = F.scaled_dot_product_attention(split(q), split(k), split(v))
    b, h, n, d = o.shape
    o = o.permute(0, 2, 1, 3).reshape(b, n, h * d)
    return _lin(o, sd, p + ".to_out.0")


# --------------------------------------------------------------------------
# UNet3DConditionModel (latentsync/models/unet.py, unet_blocks.py, resnet.py,
# attention.py, motion_module.py)
# --------------------------------------------------------------------------


def resnet_block(x, emb, sd, p, groups, eps, out_scale=1.0):
    """ResnetBlock3D.forward (resnet.py:182-223); 5-D GroupNorm (stats span frames)."""
    h = F.silu(F.group_norm(x, groups, sd[p + ".norm1.weight"], sd[p + ".norm1.bias"], eps))
    h = _inflated_conv(h, sd, p + ".conv1")
    t = _lin(F.silu(emb), sd, p + ".time_emb_proj")
    h = h + t[:, :, None, None, None]
    h = F.silu(F.group_norm(h, groups, sd[p + ".norm2.weight"], sd[p + ".norm2.bias"], eps))
    h = _inflated_conv(h, sd, p + ".conv2")
    if (p + ".conv_shortcut.weight") in sd:
        x = _inflated_conv(x, sd, p + ".conv_shortcut", padding=0)
    return (x + h) / out_scale


def transformer3d(x, audio, sd, p, heads, groups):
    """Transformer3DModel.forward (attention.py:82-124) + BasicTransformerBlock (:174-199)."""
    x4, f = _fold(x)
    bf, c, hh, ww = x4.shape
    res = x4
    h = F.group_norm(x4, groups, sd[p + ".norm.weight"], sd[p + ".norm.bias"], 1e-6)
    h = _conv(h, sd, p + ".proj_in", padding=0)
    h = h.permute(0, 2, 3, 1).reshape(bf, hh * ww, c)
    bp = p + ".transformer_blocks.0"
    h = attention(_ln(h, sd, bp + ".norm1"), sd, bp + ".attn1", heads) + h
    if (bp + ".attn2.to_q.weight") in sd and audio is not None:
        h = attention(_ln(h, sd, bp + ".norm2"), sd, bp + ".attn2", heads, context=audio) + h
    h = feed_forward(_ln(h, sd, bp + ".norm3"), sd, bp + ".ff") + h
    h = h.reshape(bf, hh, ww, c).permute(0, 3, 1, 2)
    h = _conv(h, sd, p + ".proj_out", padding=0)
    return _unfold(h + res, f)


def positional_encoding(d_model, max_len=24):
    """PositionalEncoding buffer (motion_module.py:221-230)."""
    position = torch.arange(max_len).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d_model, 2) * (-math.log(10000.0) / d_model))
    pe = torch.zeros(1, max_len, d_model)
    pe[0, :, 0::2] = torch.sin(position * div_term)
    pe[0, :, 1::2] = torch.cos(position * div_term)
    return pe


def motion_module(x, sd, p, heads, groups, max_len=24):
    """VanillaTemporalModule -> TemporalTransformer3DModel -> TemporalTransformerBlock
    -> VersatileAttention (motion_module.py:68-73, 126-151, 203-218, 262-313)."""
    tp = p + ".temporal_transformer"
    x4, f = _fold(x)
    bf, c, hh, ww = x4.shape
    res = x4
    h = F.group_norm(x4, groups, sd[tp + ".norm.weight"], sd[tp + ".norm.bias"], 1e-6)
    h = h.permute(0, 2, 3, 1).reshape(bf, hh * ww, c)
    h = _lin(h, sd, tp + ".proj_in")
    bp = tp + ".transformer_blocks.0"
    s = hh * ww
    i = 0
    while (bp + f".attention_blocks.{i}.to_q.weight") in sd:
        ap = bp + f".attention_blocks.{i}"
        n = _ln(h, sd, bp + f".norms.{i}")
        n = n.reshape(bf // f, f, s, c).permute(0, 2, 1, 3).reshape(bf // f * s, f, c)  # (b f) s c -> (b s) f c
        pe = sd.get(ap + ".pos_encoder.pe")
        if pe is None:
            pe = positional_encoding(c, max_len)
        n = n + pe[:, :f]
        a = attention(n, sd, ap, heads)
        a = a.reshape(bf // f, s, f, c).permute(0, 2, 1, 3).reshape(bf, s, c)  # (b s) f c -> (b f) s c
        h = a + h
        i += 1
    h = feed_forward(_ln(h, sd, bp + ".ff_norm"), sd, bp + ".ff") + h
    h = _lin(h, sd, tp + ".proj_out")
    h = h.reshape(bf, hh, ww, c).permute(0, 3, 1, 2)
    return _unfold(h + res, f)


def upsample_nearest(x5):
    """Upsample3D interpolation (resnet.py:53-71): nearest x2 over (h, w)."""
    return F.interpolate(x5, scale_factor=[1.0, 2.0, 2.0], mode="nearest")


def unet_forward(sd, cfg, sample, timestep, audio):
    """UNet3DConditionModel.forward (unet.py:312-471) for the configs/unet/*.yaml
    topology (unet.py:42-241).  sample (B,Cin,F,H,W) fp32, timestep an int, a float or
    a tensor of 1 or B values (broadcast over the batch, unet.py:361-376), audio
    (B*F, 50, 384) or None.  Returns (B, Cout, F, H, W)."""
    boc = list(cfg["block_out_channels"])
    nb = len(boc)
    heads = cfg.get("attention_head_dim", 8)
    heads = list(heads) if isinstance(heads, (list, tuple)) else [heads] * nb
    groups = cfg.get("norm_num_groups", 32)
    eps = float(cfg.get("norm_eps", 1e-5))
    lpb = cfg.get("layers_per_block", 2)
    mid_scale = float(cfg.get("mid_block_scale_factor", 1))
    B = sample.shape[0]
    if audio is not None and not cfg.get("add_audio_layer", False):
        audio = None

    if torch.is_tensor(timestep):
        t = timestep.reshape(-1).expand(B) if timestep.numel() == 1 else timestep.reshape(-1)
    elif isinstance(timestep, float):
        t = torch.tensor([timestep], dtype=torch.float64).expand(B)
    else:
        t = torch.full((B,), int(timestep), dtype=torch.int64)
    temb = timestep_embedding(t, boc[0], cfg.get("flip_sin_to_cos", True), cfg.get("freq_shift", 0))
    emb = _lin(F.silu(_lin(temb, sd, "time_embedding.linear_1")), sd, "time_embedding.linear_2")

    x = _inflated_conv(sample, sd, "conv_in")
    skips = [x]
    for i, btype in enumerate(cfg["down_block_types"]):
        p = f"down_blocks.{i}"
        for l in range(lpb):
            x = resnet_block(x, emb, sd, f"{p}.resnets.{l}", groups, eps)
            if btype == "CrossAttnDownBlock3D":
                x = transformer3d(x, audio, sd, f"{p}.attentions.{l}", heads[i], groups)
            if f"{p}.motion_modules.{l}.temporal_transformer.norm.weight" in sd:
                x = motion_module(x, sd, f"{p}.motion_modules.{l}", 8, groups)
            skips.append(x)
        if i < nb - 1:
            x = _inflated_conv(x, sd, f"{p}.downsamplers.0.conv", stride=2, padding=1)
            skips.append(x)

    x = resnet_block(x, emb, sd, "mid_block.resnets.0", groups, eps, mid_scale)
    x = transformer3d(x, audio, sd, "mid_block.attentions.0", heads[-1], groups)
    if "mid_block.motion_modules.0.temporal_transformer.norm.weight" in sd:
        x = motion_module(x, sd, "mid_block.motion_modules.0", 8, groups)
    x = resnet_block(x, emb, sd, "mid_block.resnets.1", groups, eps, mid_scale)

    rheads = list(reversed(heads))
    for i, btype in enumerate(cfg["up_block_types"]):
        p = f"up_blocks.{i}"
        for l in range(lpb + 1):
            x = torch.cat([x, skips.pop()], dim=1)
            x = resnet_block(x, emb, sd, f"{p}.resnets.{l}", groups, eps)
            if btype == "CrossAttnUpBlock3D":
                x = transformer3d(x, audio, sd, f"{p}.attentions.{l}", rheads[i], groups)
            if f"{p}.motion_modules.{l}.temporal_transformer.norm.weight" in sd:
                x = motion_module(x, sd, f"{p}.motion_modules.{l}", 8, groups)
        if i < nb - 1:
            x = _inflated_conv(upsample_nearest(x), sd, f"{p}.upsamplers.0.conv")

    x = F.silu(F.group_norm(x, groups, sd["conv_norm_out.weight"], sd["conv_norm_out.bias"], eps))
    return _inflated_conv(x, sd, "conv_out")


# --------------------------------------------------------------------------
# SD AutoencoderKL (diffusers 0.32.2 restated; unpinned)
# --------------------------------------------------------------------------

VAE_CFG = dict(block_out_channels=(128, 256, 512, 512), layers_per_block=2, groups=32, eps=1e-6,
               latent_channels=4, scaling_factor=0.18215, shift_factor=0.0)


def _vae_resnet(x, sd, p, groups=32, eps=1e-6):
    h = F.silu(F.group_norm(x, groups, sd[p + ".norm1.weight"], sd[p + ".norm1.bias"], eps))
    h = _conv(h, sd, p + ".conv1")
    h = F.silu(F.group_norm(h, groups, sd[p + ".norm2.weight"], sd[p + ".norm2.bias"], eps))
    h = _conv(h, sd, p + ".conv2")
    if (p + ".conv_shortcut.weight") in sd:
        x = _conv(x, sd, p + ".conv_shortcut", padding=0)
    return x + h


def _vae_attn(x, sd, p, groups=32, eps=1e-6):
    b, c, hh, ww = x.shape
    res = x
    h = F.group_norm(x, groups, sd[p + ".group_norm.weight"], sd[p + ".group_norm.bias"], eps)
    h = h.reshape(b, c, hh * ww).transpose(1, 2)
    q, k, v = (_lin(h, sd, p + n) for n in (".to_q", ".to_k", ".to_v"))
    o = F.scaled_dot_product_attention(q[:, None], k[:, None], v[:, None])[:, 0]
    o = _lin(o, sd, p + ".to_out.0")
    return o.transpose(1, 2).reshape(b, c, hh, ww) + res


def _vae_mid(x, sd, p):
    x = _vae_resnet(x, sd, p + ".resnets.0")
    x = _vae_attn(x, sd, p + ".attentions.0")
    return _vae_resnet(x, sd, p + ".resnets.1")


def vae_encode_moments(sd, x):
    """AutoencoderKL.encode -> quant_conv moments (N, 8, H/8, W/8)."""
    boc = VAE_CFG["block_out_channels"]
    h = _conv(x, sd, "encoder.conv_in")
    for i in range(len(boc)):
        for l in range(VAE_CFG["layers_per_block"]):
            h = _vae_resnet(h, sd, f"encoder.down_blocks.{i}.resnets.{l}")
        if i < len(boc) - 1:
            h = F.pad(h, (0, 1, 0, 1))
            h = _conv(h, sd, f"encoder.down_blocks.{i}.downsamplers.0.conv", stride=2, padding=0)
    h = _vae_mid(h, sd, "encoder.mid_block")
    h = F.silu(F.group_norm(h, 32, sd["encoder.conv_norm_out.weight"], sd["encoder.conv_norm_out.bias"], 1e-6))
    h = _conv(h, sd, "encoder.conv_out")
    return _conv(h, sd, "quant_conv", padding=0)


def vae_sample(moments, eps_noise):
    """DiagonalGaussianDistribution(moments).sample() with injected noise."""
    mean, logvar = moments.chunk(2, dim=1)
    logvar = torch.clamp(logvar, -30.0, 20.0)
    return mean + torch.exp(0.5 * logvar) * eps_noise


def vae_decode(sd, z):
    """AutoencoderKL.decode(z).sample."""
    boc = list(reversed(VAE_CFG["block_out_channels"]))
    h = _conv(z, sd, "post_quant_conv", padding=0)
    h = _conv(h, sd, "decoder.conv_in")
    h = _vae_mid(h, sd, "decoder.mid_block")
    for i in range(len(boc)):
        for l in range(VAE_CFG["layers_per_block"] + 1):
            h = _vae_resnet(h, sd, f"decoder.up_blocks.{i}.resnets.{l}")
        if i < len(boc) - 1:
            h = F.interpolate(h, scale_factor=2.0, mode="nearest")
            h = _conv(h, sd, f"decoder.up_blocks.{i}.upsamplers.0.conv")
    h = F.silu(F.group_norm(h, 32, sd["decoder.conv_norm_out.weight"], sd["decoder.conv_norm_out.bias"], 1e-6))
    return _conv(h, sd, "decoder.conv_out")


# --------------------------------------------------------------------------
# DDIMScheduler (diffusers 0.32.2 restated; configs/scheduler_config.json)
# --------------------------------------------------------------------------


def ddim_alphas_cumprod(beta_start=0.00085, beta_end=0.012, T=1000):
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, T, dtype=torch.float32) ** 2
    return torch.cumprod(1.0 - betas, dim=0)


def ddim_timesteps(n, T=1000, steps_offset=1):
    ratio = T // n
    return (np.arange(0, n) * ratio).round()[::-1].copy().astype(np.int64) + steps_offset


def ddim_step(ac, eps, t, x, n, T=1000):
    """DDIMScheduler.step, eta=0, epsilon prediction, no clipping."""
    prev = t - T // n
    a_t = ac[t]
    a_p = ac[prev] if prev >= 0 else ac[0]
    x0 = (x - (1 - a_t) ** 0.5 * eps) / a_t ** 0.5
    return a_p ** 0.5 * x0 + (1 - a_p) ** 0.5 * eps


# --------------------------------------------------------------------------
# Whisper-tiny audio features (latentsync/whisper/*)
# --------------------------------------------------------------------------


def whisper_sinusoids(length, channels, max_timescale=10000):
    """whisper/model.py:48-54."""
    inc = np.log(max_timescale) / (channels // 2 - 1)
    inv = torch.exp(-inc * torch.arange(channels // 2))
    st = torch.arange(length)[:, None] * inv[None, :]
    return torch.cat([torch.sin(st), torch.cos(st)], dim=1)


def whisper_encoder_layers(sd, mel, n_head=6):
    """AudioEncoder.forward(include_embeddings=True) (whisper/model.py:143-171):
    mel (1, 80, 3000) -> (1, 5, 1500, 384) stack of [post-pos-emb, block1..block4]."""
    x = F.gelu(F.conv1d(mel, sd["encoder.conv1.weight"], sd["encoder.conv1.bias"], padding=1))
    x = F.gelu(F.conv1d(x, sd["encoder.conv2.weight"], sd["encoder.conv2.bias"], stride=2, padding=1))
    x = x.permute(0, 2, 1)
    x = x + whisper_sinusoids(x.shape[1], x.shape[2])
    outs = [x]
    i = 0
    while f"encoder.blocks.{i}.attn.query.weight" in sd:
        p = f"encoder.blocks.{i}"
        h = _ln(x, sd, p + ".attn_ln")
        q = _lin(h, sd, p + ".attn.query")
        k = _lin(h, sd, p + ".attn.key", bias=False)
        v = _lin(h, sd, p + ".attn.value")
        b, n, c = q.shape
        d = c // n_head
        s = d ** -0.25
        q = q.view(b, n, n_head, d).permute(0, 2, 1, 3) * s
        k = k.view(b, n, n_head, d).permute(0, 2, 3, 1) * s
        v = v.view(b, n, n_head, d).permute(0, 2, 1, 3)
        w = torch.softmax((q @ k).float(), dim=-1)
        o = (w @ v).permute(0, 2, 1, 3).flatten(start_dim=2)
        x = x + _lin(o, sd, p + ".attn.out")
        h = _ln(x, sd, p + ".mlp_ln")
        x = x + _lin(F.gelu(_lin(h, sd, p + ".mlp.0")), sd, p + ".mlp.2")
        outs.append(x)
        i += 1
    return torch.stack(outs, dim=1)


def log_mel_spectrogram(audio, filters):
    """whisper/audio.py:92-125 for an in-memory 16 kHz waveform."""
    audio = torch.as_tensor(audio, dtype=torch.float32)
    window = torch.hann_window(400)
    stft = torch.stft(audio, 400, 160, window=window, return_complex=True)
    mag = stft[:, :-1].abs() ** 2
    mel = torch.as_tensor(filters) @ mag
    log_spec = torch.clamp(mel, min=1e-10).log10()
    log_spec = torch.maximum(log_spec, log_spec.max() - 8.0)
    return (log_spec + 4.0) / 4.0


def whisper_features(sd, audio, filters):
    """Audio2Feature._audio2feat (audio2feature.py:102-115) + transcribe's segment
    loop (transcribe.py:85-128): 3000-frame mel segments, keep (end-start)//2 rows."""
    mel = log_mel_spectrogram(audio, filters)
    n = mel.shape[-1]
    feats = []
    seek = 0
    while seek < n:
        end = min(seek + 3000, n)
        seg = mel[:, seek:seek + 3000]
        seg = F.pad(seg, (0, 3000 - seg.shape[-1]))
        emb = whisper_encoder_layers(sd, seg[None])[0]  # (5, 1500, 384)
        emb = emb.permute(1, 0, 2)
        feats.append(emb[: int((end - seek) / 2)])
        seek += 3000
    return torch.cat(feats, dim=0)


def sliced_feature_index(length, vid_idx, fps=25, feat_len=(2, 2)):
    """get_sliced_feature's index list (audio2feature.py:24-49)."""
    center = int(vid_idx * 50 / fps)
    left = center - feat_len[0] * 2
    right = center + (feat_len[1] + 1) * 2
    return [min(length - 1, max(0, i)) for i in range(left, right)]


def feature2chunks(feature, fps=25, feat_len=(2, 2)):
    """Audio2Feature.feature2chunks (audio2feature.py:85-100)."""
    out = []
    i = 0
    mult = 50.0 / fps
    T = len(feature)
    emb = feature.shape[-1]
    while True:
        start = int(i * mult)
        idx = sliced_feature_index(T, i, fps, feat_len)
        out.append(feature[idx].reshape(-1, emb))
        i += 1
        if start > T:
            break
    return out


# --------------------------------------------------------------------------
# Pipeline window (lipsync_pipeline.py:500-575), with injected noise
# --------------------------------------------------------------------------


def prepare_pixels(faces_u8, mask):
    """ImageProcessor.preprocess_fixed_mask_image (image_processor.py:145-152) at
    native resolution (Resize is the identity there).  faces (F,3,R,R) uint8,
    mask (R,R) float in {0,1} (1 = keep).  Returns pixel, masked, mask(F,1,R,R)."""
    pix = (faces_u8.to(torch.float32) / 255.0 - 0.5) / 0.5
    m = mask.to(torch.float32)
    masked = pix * m
    return pix, masked, m.expand(pix.shape[0], 1, *m.shape)


def pipeline_window(unet_sd, unet_cfg, vae_sd, faces_u8, mask, audio_chunks, init_latent, eps_masked, eps_ref,
                    num_steps=20, guidance_scale=1.0, step_latents=None):
    """One 16-frame window of LipsyncPipeline.__call__ (lipsync_pipeline.py:500-575).
    faces_u8 (F,3,R,R); mask (R,R) 1=keep; audio_chunks (F,50,384);
    init_latent (1,4,1,h,w) repeated over frames (prepare_latents :182-196);
    eps_* (F,4,h,w) the VAE posterior noise.  Returns decoded+pasted (F,3,R,R).
    ``step_latents``: a list that receives the (1,4,F,h,w) latents after every DDIM
    step -- what the reference hands its callback (:562-568)."""
    Fn = faces_u8.shape[0]
    cfg_on = guidance_scale > 1.0
    pix, masked, m = prepare_pixels(faces_u8, mask)
    h = pix.shape[-1] // 8
    sc = VAE_CFG["scaling_factor"]
    mask_lat = F.interpolate(m, size=(h, h))                                  # :290-292
    masked_lat = vae_sample(vae_encode_moments(vae_sd, masked), eps_masked) * sc  # :296-297
    ref_lat = vae_sample(vae_encode_moments(vae_sd, pix), eps_ref) * sc           # :315-316
    to5 = lambda t: t.permute(1, 0, 2, 3)[None]  # "f c h w -> 1 c f h w"
    mask_lat, masked_lat, ref_lat = to5(mask_lat), to5(masked_lat), to5(ref_lat)
    audio = audio_chunks
    if cfg_on:
        mask_lat, masked_lat, ref_lat = (torch.cat([t, t]) for t in (mask_lat, masked_lat, ref_lat))
        audio = torch.cat([torch.zeros_like(audio), audio])
    lat = init_latent.repeat(1, 1, Fn, 1, 1)
    ac = ddim_alphas_cumprod()
    for t in ddim_timesteps(num_steps):
        inp = torch.cat([lat] * 2) if cfg_on else lat
        inp = torch.cat([inp, mask_lat, masked_lat, ref_lat], dim=1)
        eps = unet_forward(unet_sd, unet_cfg, inp, int(t), audio)
        if cfg_on:
            u, a = eps.chunk(2)
            eps = u + guidance_scale * (a - u)
        lat = ddim_step(ac, eps, int(t), lat, num_steps)
        if step_latents is not None:
            step_latents.append(lat.clone())
    z = lat / sc                                                                 # decode_latents :145-149
    z = z[0].permute(1, 0, 2, 3)
    dec = vae_decode(vae_sd, z)
    keep = m
    return dec * (1 - keep) + pix * keep                                          # paste-back :327-333, :572-574
