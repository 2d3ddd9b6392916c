"""State-dict key/shape schemas of the three networks on the hot path.

The loader accepts checkpoints with exactly the reference's key names
(SURVEY.md Appendix B), so the schema mirrors the module construction of
  * UNet3DConditionModel: latentsync/models/unet.py:85-241 + unet_blocks.py
    (CrossAttnDownBlock3D :263-357, DownBlock3D :410-476, UNetMidBlock3DCrossAttn
    :153-245, CrossAttnUpBlock3D :519-609, UpBlock3D :669-731), resnet.py:104-180,
    attention.py:15-185, motion_module.py:39-257;
  * diffusers AutoencoderKL (sd-vae-ft-mse layout);
  * whisper AudioEncoder (latentsync/whisper/whisper/model.py:103-141).
"""
from collections import OrderedDict


def _norm(sd, p, c):
    sd[p + ".weight"] = (c,)
    sd[p + ".bias"] = (c,)


def _lin(sd, p, o, i, bias=True):
    sd[p + ".weight"] = (o, i)
    if bias:
        sd[p + ".bias"] = (o,)


def _conv(sd, p, o, i, k):
    sd[p + ".weight"] = (o, i, k, k)
    sd[p + ".bias"] = (o,)


def _resnet(sd, p, cin, cout, temb=1280):
    _norm(sd, p + ".norm1", cin)
    _conv(sd, p + ".conv1", cout, cin, 3)
    if temb:
        _lin(sd, p + ".time_emb_proj", cout, temb)
    _norm(sd, p + ".norm2", cout)
    _conv(sd, p + ".conv2", cout, cout, 3)
    if cin != cout:
        _conv(sd, p + ".conv_shortcut", cout, cin, 1)


def _ff(sd, p, c):
    _lin(sd, p + ".net.0.proj", 8 * c, c)
    _lin(sd, p + ".net.2", c, 4 * c)


def _transformer(sd, p, c, cross_dim, audio):
    _norm(sd, p + ".norm", c)
    _conv(sd, p + ".proj_in", c, c, 1)
    b = p + ".transformer_blocks.0"
    _norm(sd, b + ".norm1", c)
    for n in ("to_q", "to_k", "to_v"):
        _lin(sd, f"{b}.attn1.{n}", c, c, bias=False)
    _lin(sd, b + ".attn1.to_out.0", c, c)
    if audio:
        _norm(sd, b + ".norm2", c)
        _lin(sd, b + ".attn2.to_q", c, c, bias=False)
        _lin(sd, b + ".attn2.to_k", c, cross_dim, bias=False)
        _lin(sd, b + ".attn2.to_v", c, cross_dim, bias=False)
        _lin(sd, b + ".attn2.to_out.0", c, c)
    _ff(sd, b + ".ff", c)
    _norm(sd, b + ".norm3", c)
    _conv(sd, p + ".proj_out", c, c, 1)


def _motion(sd, p, c, kw):
    t = p + ".temporal_transformer"
    _norm(sd, t + ".norm", c)
    _lin(sd, t + ".proj_in", c, c)
    b = t + ".transformer_blocks.0"
    for i, _ in enumerate(kw.get("attention_block_types", ("Temporal_Self", "Temporal_Self"))):
        a = f"{b}.attention_blocks.{i}"
        for n in ("to_q", "to_k", "to_v"):
            _lin(sd, f"{a}.{n}", c, c, bias=False)
        _lin(sd, a + ".to_out.0", c, c)
        if kw.get("temporal_position_encoding", False):
            sd[a + ".pos_encoder.pe"] = (1, kw.get("temporal_position_encoding_max_len", 24), c)
    for i, _ in enumerate(kw.get("attention_block_types", ("Temporal_Self", "Temporal_Self"))):
        _norm(sd, f"{b}.norms.{i}", c)
    _ff(sd, b + ".ff", c)
    _norm(sd, b + ".ff_norm", c)
    _lin(sd, t + ".proj_out", c, c)


def unet_param_shapes(cfg: dict) -> "OrderedDict[str, tuple]":
    boc = list(cfg["block_out_channels"])
    nb = len(boc)
    lpb = cfg.get("layers_per_block", 2)
    temb = boc[0] * 4
    cross = cfg.get("cross_attention_dim", 1280)
    audio = cfg.get("add_audio_layer", False)
    mm = cfg.get("use_motion_module", False)
    mres = cfg.get("motion_module_resolutions", (1, 2, 4, 8))
    mkw = cfg.get("motion_module_kwargs", {}) or {}
    sd = OrderedDict()
    _conv(sd, "conv_in", boc[0], cfg["in_channels"], 3)
    _lin(sd, "time_embedding.linear_1", temb, boc[0])
    _lin(sd, "time_embedding.linear_2", temb, temb)
    out_c = boc[0]
    for i, bt in enumerate(cfg["down_block_types"]):
        in_c, out_c = out_c, boc[i]
        p = f"down_blocks.{i}"
        use_mm = mm and (2 ** i in mres) and not cfg.get("motion_module_decoder_only", False)
        for l in range(lpb):
            _resnet(sd, f"{p}.resnets.{l}", in_c if l == 0 else out_c, out_c, temb)
            if bt == "CrossAttnDownBlock3D":
                _transformer(sd, f"{p}.attentions.{l}", out_c, cross, audio)
            if use_mm:
                _motion(sd, f"{p}.motion_modules.{l}", out_c, mkw)
        if i < nb - 1:
            _conv(sd, f"{p}.downsamplers.0.conv", out_c, out_c, 3)
    c = boc[-1]
    _resnet(sd, "mid_block.resnets.0", c, c, temb)
    _transformer(sd, "mid_block.attentions.0", c, cross, audio)
    if mm and cfg.get("motion_module_mid_block", False):
        _motion(sd, "mid_block.motion_modules.0", c, mkw)
    _resnet(sd, "mid_block.resnets.1", c, c, temb)
    rev = list(reversed(boc))
    out_c = rev[0]
    for i, bt in enumerate(cfg["up_block_types"]):
        prev_c, out_c = out_c, rev[i]
        in_c = rev[min(i + 1, nb - 1)]
        p = f"up_blocks.{i}"
        use_mm = mm and (2 ** (3 - i) in mres)
        for l in range(lpb + 1):
            skip_c = in_c if l == lpb else out_c
            r_in = prev_c if l == 0 else out_c
            _resnet(sd, f"{p}.resnets.{l}", r_in + skip_c, out_c, temb)
            if bt == "CrossAttnUpBlock3D":
                _transformer(sd, f"{p}.attentions.{l}", out_c, cross, audio)
            if use_mm:
                _motion(sd, f"{p}.motion_modules.{l}", out_c, mkw)
        if i < nb - 1:
            _conv(sd, f"{p}.upsamplers.0.conv", out_c, out_c, 3)
    _norm(sd, "conv_norm_out", boc[0])
    _conv(sd, "conv_out", cfg["out_channels"], boc[0], 3)
    return sd


def vae_param_shapes(boc=(128, 256, 512, 512), lpb=2, latent=4) -> "OrderedDict[str, tuple]":
    sd = OrderedDict()

    def mid(p, c):
        _resnet(sd, p + ".resnets.0", c, c, 0)
        a = p + ".attentions.0"
        _norm(sd, a + ".group_norm", c)
        for n in ("to_q", "to_k", "to_v", "to_out.0"):
            _lin(sd, f"{a}.{n}", c, c)
        _resnet(sd, p + ".resnets.1", c, c, 0)

    _conv(sd, "encoder.conv_in", boc[0], 3, 3)
    out_c = boc[0]
    for i in range(len(boc)):
        in_c, out_c = out_c, boc[i]
        for l in range(lpb):
            _resnet(sd, f"encoder.down_blocks.{i}.resnets.{l}", in_c if l == 0 else out_c, out_c, 0)
        if i < len(boc) - 1:
            _conv(sd, f"encoder.down_blocks.{i}.downsamplers.0.conv", out_c, out_c, 3)
    mid("encoder.mid_block", boc[-1])
    _norm(sd, "encoder.conv_norm_out", boc[-1])
    _conv(sd, "encoder.conv_out", 2 * latent, boc[-1], 3)
    _conv(sd, "quant_conv", 2 * latent, 2 * latent, 1)
    _conv(sd, "post_quant_conv", latent, latent, 1)
    rev = list(reversed(boc))
    _conv(sd, "decoder.conv_in", rev[0], latent, 3)
    mid("decoder.mid_block", rev[0])
    out_c = rev[0]
    for i in range(len(rev)):
        prev_c, out_c = out_c, rev[i]
        for l in range(lpb + 1):
            _resnet(sd, f"decoder.up_blocks.{i}.resnets.{l}", prev_c if l == 0 else out_c, out_c, 0)
        if i < len(rev) - 1:
            _conv(sd, f"decoder.up_blocks.{i}.upsamplers.0.conv", out_c, out_c, 3)
    _norm(sd, "decoder.conv_norm_out", rev[-1])
    _conv(sd, "decoder.conv_out", 3, rev[-1], 3)
    return sd


def whisper_encoder_param_shapes(n_mels=80, n_ctx=1500, n_state=384, n_layer=4) -> "OrderedDict[str, tuple]":
    sd = OrderedDict()
    sd["encoder.conv1.weight"] = (n_state, n_mels, 3)
    sd["encoder.conv1.bias"] = (n_state,)
    sd["encoder.conv2.weight"] = (n_state, n_state, 3)
    sd["encoder.conv2.bias"] = (n_state,)
    sd["encoder.positional_embedding"] = (n_ctx, n_state)
    for i in range(n_layer):
        p = f"encoder.blocks.{i}"
        _lin(sd, p + ".attn.query", n_state, n_state)
        _lin(sd, p + ".attn.key", n_state, n_state, bias=False)
        _lin(sd, p + ".attn.value", n_state, n_state)
        _lin(sd, p + ".attn.out", n_state, n_state)
        _norm(sd, p + ".attn_ln", n_state)
        _lin(sd, p + ".mlp.0", 4 * n_state, n_state)
        _lin(sd, p + ".mlp.2", n_state, 4 * n_state)
        _norm(sd, p + ".mlp_ln", n_state)
    _norm(sd, "encoder.ln_post", n_state)
    return sd
