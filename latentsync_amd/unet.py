"""UNet3DConditionModel -- MI355X-native drop-in for
latentsync/models/unet.py:39-512.

Same constructor kwargs (the configs/unet/*.yaml ``model:`` schema), same
``from_pretrained(model_config, ckpt_path, device)`` / ``load_state_dict`` drop
rules / ``forward(sample, timestep, encoder_hidden_states, ...)`` signature and
``UNet3DConditionOutput(sample=...)`` result.  Underneath, every op runs in the
HIP C-ABI library (latentsync_amd/ops.py -> libls_hip.so) on NHWC bf16
activations with frames folded into the image index:

  ResnetBlock3D (resnet.py:182-223)
      GN5D stats -> GN-apply+SiLU -> conv1 3x3 [bias + temb epilogue]
      GN5D stats -> GN-apply+SiLU -> conv2 3x3 [bias + shortcut residual]
      the up-block torch.cat (unet_blocks.py:624,745) is fused into the gathers.
  Transformer3DModel (attention.py:82-124) + BasicTransformerBlock (:174-199)
      GN4D stats -> GN-apply -> proj_in 1x1 -> LN -> fused q|k|v GEMM ->
      flash attention -> out-proj [bias + residual] -> LN -> q GEMM, audio k|v
      GEMM -> attention (Nk = 50) -> out-proj -> LN -> GEGLU GEMM (fused
      h * gelu(g) epilogue) -> FF2 [bias + residual] -> proj_out [+ residual]
  VanillaTemporalModule (motion_module.py:39-313)
      GN4D -> GN-apply -> proj_in -> 2 x (LN + pos-enc -> q|k|v -> temporal
      attention over frames via strided views -> out-proj) -> GEGLU FF -> proj_out
"""
import math
from dataclasses import dataclass

import torch

from . import _lib, ops
from .config import STAGE2_MODEL
from .packing import geglu_interleave, pack_ff_w2, pack_weight, pad_bias
from .schema import unet_param_shapes
from .weights import fill_state_dict

# A/B switches (read from the environment only in diagnostics mode, _lib.ab_switch):
# LS_FUSED_TEMPORAL=0: the motion attention as q|k|v GEMM + ls_attention
_FUSED_TEMPORAL = _lib.ab_switch("LS_FUSED_TEMPORAL", "1") != "0"
# LS_FUSED_FF=0: the FeedForward as GEGLU row-block GEMM + W2 GEMM
_FUSED_FF = _lib.ab_switch("LS_FUSED_FF", "1") != "0"
# LS_FF_CHAIN=0: the 32x32-level block tail (to_out + LN + FeedForward + proj_out) as three
# launches (row-block GEMM, ls_feedforward, row-block GEMM) instead of one ls_ff_chain
_FF_CHAIN = _lib.ab_switch("LS_FF_CHAIN", "1") != "0"
# conv_norm_out + SiLU + conv_out on the narrow halo tile, conv_out padded to 8 columns (round 6;
# "0" in diagnostics mode: the materialised GroupNorm and the 4-column tiled GEMM)
_NARROW_OUT = _lib.ab_switch("LS_NARROW_OUT", "1") != "0"
# LS_FUSED_XATTN=1: the audio cross-attention branch at C = 320 as ONE ls_cross_attention_block
# launch instead of q GEMM + ls_attention + out GEMM.  Off by default: measured 1-2 ms per
# 48-window step SLOWER than the three launches (profiles/r04k_step_ab.txt)
_FUSED_XATTN = _lib.ab_switch("LS_FUSED_XATTN", "0") == "1"


def _ff(h, st, ff1, ff2, ff2p):
    """norm + FeedForward + residual: ls_feedforward at C = 320 (the GEGLU intermediate
    stays in registers), else the GEGLU GEMM (LN folded) and the W2 GEMM with the residual."""
    if ff2p is not None and ops.feedforward_ok(h, ff1, ff2):
        return ops.feedforward(h, st, ff1, ff2, ff2p)
    g = ops.linear(h, ff1, act=ops.ACT_GEGLU, ln_stats=st)
    return ops.linear(g, ff2, res=h)


def _chain_pack(o, ff1, ff2, po, c):
    """ls_ff_chain operands of a C = 320 block tail (ops.pack_ff_chain), or None."""
    if not (_FF_CHAIN and _FUSED_FF and c == 320 and ff1.N == 2560 and ff2.N == 320 and ff2.K == 1280):
        return None
    return ops.pack_ff_chain(o, ff1, ff2, po)


def _ff2_packed(dv, key):
    """W2 of a C = 320 FeedForward re-packed for ls_feedforward (packing.pack_ff_w2)."""
    w = dv.sd[key]
    if not _FUSED_FF or tuple(w.shape) != (320, 1280):
        return None
    return pack_ff_w2(w.float().cpu()).to(torch.bfloat16).to(dv.device).contiguous()

_DEFAULTS = dict(
    sample_size=None, in_channels=4, out_channels=4, center_input_sample=False, flip_sin_to_cos=True, freq_shift=0,
    down_block_types=("CrossAttnDownBlock3D", "CrossAttnDownBlock3D", "CrossAttnDownBlock3D", "DownBlock3D"),
    mid_block_type="UNetMidBlock3DCrossAttn",
    up_block_types=("UpBlock3D", "CrossAttnUpBlock3D", "CrossAttnUpBlock3D", "CrossAttnUpBlock3D"),
    only_cross_attention=False, block_out_channels=(320, 640, 1280, 1280), layers_per_block=2, downsample_padding=1,
    mid_block_scale_factor=1, act_fn="silu", norm_num_groups=32, norm_eps=1e-5, cross_attention_dim=1280,
    attention_head_dim=8, dual_cross_attention=False, use_linear_projection=False, class_embed_type=None,
    num_class_embeds=None, upcast_attention=False, resnet_time_scale_shift="default", use_inflated_groupnorm=False,
    use_motion_module=False, motion_module_resolutions=(1, 2, 4, 8), motion_module_mid_block=False,
    motion_module_decoder_only=False, motion_module_type=None, motion_module_kwargs={}, add_audio_layer=False,
)


class FrozenDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


@dataclass
class UNet3DConditionOutput:
    sample: torch.Tensor

    def __getitem__(self, i):
        return (self.sample,)[i]


def positional_encoding(d_model, max_len=24):
    """PositionalEncoding buffer (motion_module.py:221-230)."""
    position = torch.arange(max_len).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d_model, 2) * (-math.log(10000.0) / d_model))
    pe = torch.zeros(max_len, d_model)
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe


# --------------------------------------------------------------------------
# packed device-side layers
# --------------------------------------------------------------------------


class _Dev:
    def __init__(self, sd, device):
        self.sd, self.device = sd, device

    def f32(self, key):
        return self.sd[key].float().to(self.device).contiguous()

    def packed(self, wkey, bkey=None, ksize=None, cin_pad=None, n_pad=None, w=None, b=None, geglu=False):
        w = self.sd[wkey] if w is None else w
        b = (self.sd.get(bkey) if bkey else None) if b is None else b
        if ksize is None:
            ksize = w.shape[-1] if w.dim() == 4 else 1
        n_out = max(w.shape[0], n_pad or 0)  # padded output channels are written as zeros
        if geglu:
            w, b = geglu_interleave(w.float(), b.float())
        wp = pack_weight(w, cin_pad=cin_pad, n_pad=n_pad)
        bp = pad_bias(b, n_pad)
        cin = cin_pad or (w.shape[1] + 7) // 8 * 8
        return ops.Packed(wp.to(torch.bfloat16).to(self.device).contiguous(),
                          None if bp is None else bp.to(self.device).contiguous(), cin, ksize, n_out, geglu)

    def packed_ln(self, w, b, ln, geglu=False, pe=None):
        """nn.LayerNorm(gamma, beta) followed by linear(w, b), folded for the GEMM
        epilogue (ls_conv_desc.ln_rowstats): Wp = W * gamma, bias = b + W beta,
        colsum = row sums of the packed bf16 Wp; with a positional encoding added
        after the norm (motion_module.py:267), pe_rows = pe W^T (rowvec table)."""
        gamma, beta = (t.detach().float().cpu() for t in ln)
        w = w.float().cpu()
        b = (b.float().cpu() if b is not None else torch.zeros(w.shape[0])) + w @ beta
        pk = self.packed(None, w=w * gamma[None, :], b=b, geglu=geglu)
        pk.colsum = pk.w.float().sum(1).contiguous()
        if pe is not None:
            pk.pe_rows = (pe.float().cpu() @ w.T).to(self.device).contiguous()
        return pk


class _Resnet:
    def __init__(self, dv, p, cin, cout, groups, eps, out_scale, temb_slot):
        self.groups, self.eps, self.cin, self.cout = groups, eps, cin, cout
        self.n1 = (dv.f32(p + ".norm1.weight"), dv.f32(p + ".norm1.bias"))
        self.n2 = (dv.f32(p + ".norm2.weight"), dv.f32(p + ".norm2.bias"))
        self.c1 = dv.packed(p + ".conv1.weight", p + ".conv1.bias")
        self.c2 = dv.packed(p + ".conv2.weight", p + ".conv2.bias")
        self.sc = dv.packed(p + ".conv_shortcut.weight", p + ".conv_shortcut.bias") \
            if (p + ".conv_shortcut.weight") in dv.sd else None
        self.out_scale = 1.0 / out_scale
        self.temb_slot = temb_slot  # column offset into the batched temb projection

    def __call__(self, x, B, temb_all, x2=None):
        n = x.shape[0]
        F = n // B
        pps = F * x.shape[1] * x.shape[2]
        s1 = ops.group_norm(x, self.groups, self.eps, *self.n1, B, x2=x2)
        # GN affine + SiLU: applied once per pixel in the halo-tile conv's LDS image where it
        # takes the call (ls_conv_path 3: 32x32 / 16x16), else materialised (ops.conv)
        # gn_out: GroupNorm statistics of every GN input come from its producer's epilogue
        # temb_all: one row per sample, or ONE row for the whole batch (_DeviceUNet.temb, the
        # UNet forward: one timestep) -- then rows_per_vec spans all rows
        rpv = pps * B if temb_all.shape[0] == 1 else pps
        h = ops.conv(x, self.c1, x2=x2, aff=(s1[0], s1[1], F, True), aff_materialize=True,
                     rowvec=(temb_all[:, self.temb_slot:], rpv, temb_all.shape[1]), gn_out=True)
        s2 = ops.group_norm(h, self.groups, self.eps, *self.n2, B)
        res = x if self.sc is None else ops.conv(x, self.sc, x2=x2)
        return ops.conv(h, self.c2, aff=(s2[0], s2[1], F, True), aff_materialize=True, res=res,
                        out_scale=self.out_scale, gn_out=True)


class _Transformer:
    def __init__(self, dv, p, c, heads, groups, audio):
        self.c, self.heads, self.groups = c, heads, groups
        self.fp8 = False  # spatial self attention's P V on the fp8 MFMA (configs[4])
        self.norm = (dv.f32(p + ".norm.weight"), dv.f32(p + ".norm.bias"))
        self.proj_in = dv.packed(p + ".proj_in.weight", p + ".proj_in.bias")
        self.proj_out = dv.packed(p + ".proj_out.weight", p + ".proj_out.bias")
        b = p + ".transformer_blocks.0"
        sd = dv.sd
        ln = lambda k: (sd[k + ".weight"], sd[k + ".bias"])
        self.qkv1 = dv.packed_ln(torch.cat([sd[f"{b}.attn1.to_{n}.weight"] for n in "qkv"], 0), None, ln(b + ".norm1"))
        self.o1 = dv.packed(b + ".attn1.to_out.0.weight", b + ".attn1.to_out.0.bias")
        self.has_audio = audio and (b + ".attn2.to_q.weight") in sd
        if self.has_audio:
            self.q2 = dv.packed_ln(sd[b + ".attn2.to_q.weight"], None, ln(b + ".norm2"))
            self.kv2 = dv.packed(None, w=torch.cat([sd[b + ".attn2.to_k.weight"], sd[b + ".attn2.to_v.weight"]], 0))
            self.o2 = dv.packed(b + ".attn2.to_out.0.weight", b + ".attn2.to_out.0.bias")
            # norm2 + to_q + SDPA + to_out + residual in one launch at C = 320 (ls_cross_attention_block)
            self.xa = ops.pack_cross_attention(
                sd[b + ".attn2.to_q.weight"], *ln(b + ".norm2"), sd[b + ".attn2.to_out.0.weight"],
                sd[b + ".attn2.to_out.0.bias"], heads, dv.device) if _FUSED_XATTN and c == 320 and heads == 8 else None
        self.ff1 = dv.packed_ln(sd[b + ".ff.net.0.proj.weight"], sd[b + ".ff.net.0.proj.bias"], ln(b + ".norm3"),
                                geglu=True)
        self.ff2 = dv.packed(b + ".ff.net.2.weight", b + ".ff.net.2.bias")
        self.ff2p = _ff2_packed(dv, b + ".ff.net.2.weight")
        # attn2.to_out + norm3 + ff + proj_out in one launch at C = 320 (ls_ff_chain)
        self.chain = _chain_pack(self.o2, self.ff1, self.ff2, self.proj_out, c) if self.has_audio else None

    def audio_kv(self, audio_rows):
        """The audio cross-attention k|v projection (attn2.to_k / to_v of the audio
        embeddings).  It does not depend on the latents, so the window engine computes it
        once per batch of windows instead of once per DDIM step."""
        return ops.linear(audio_rows, self.kv2) if self.has_audio else None

    def __call__(self, x, audio_rows, n_audio_tok, kv=None):
        n, H, W, C = x.shape
        HW = H * W
        rows = n * HW
        d = C // self.heads
        sc = ops.group_norm(x, self.groups, 1e-6, *self.norm, n)
        # LayerNorm statistics of every h come out of the GEMM that writes h
        st = torch.empty((rows, 2), dtype=torch.float32, device=x.device)
        # GN affine folded into the row-block GEMM's A rows (32x32 / 16x16); materialised elsewhere
        h = ops.conv(x, self.proj_in, aff=(sc[0], sc[1], 1, False), aff_materialize=True,
                     stats_out=st).view(rows, C)
        # self attention (norm1 folded into the q|k|v GEMM)
        qkv = ops.linear(h, self.qkv1, ln_stats=st)
        o = torch.empty((rows, C), dtype=torch.bfloat16, device=x.device)
        ops.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=n, z2=1, heads=self.heads, nq=HW, nk=HW, head_dim=d,
                      qs=(HW * 3 * C, 0, 3 * C, d), ks=(HW * 3 * C, 0, 3 * C, d), vs=(HW * 3 * C, 0, 3 * C, d),
                      os_=(HW * C, 0, C, d), fp8=self.fp8 and HW > 128 and d in (40, 80))
        h = ops.linear(o, self.o1, res=h, stats_out=st)
        # audio cross attention
        if self.has_audio and audio_rows is not None:
            if kv is None:
                kv = ops.linear(audio_rows, self.kv2)
            L = n_audio_tok
            if ops.cross_attention_ok(h, self.xa, L, HW):
                st2 = torch.empty_like(st)
                h = ops.cross_attention_block(h, st, self.xa, kv, L, HW, st2)
                st = st2
                return self._tail(x, h, st, n, H, W, C)
            q = ops.linear(h, self.q2, ln_stats=st)
            ops.attention(q, kv, kv[:, C:], o, batch=n, z2=1, heads=self.heads, nq=HW, nk=L, head_dim=d,
                          qs=(HW * C, 0, C, d), ks=(L * 2 * C, 0, 2 * C, d), vs=(L * 2 * C, 0, 2 * C, d),
                          os_=(HW * C, 0, C, d))
            if ops.ff_chain_ok(o, self.chain):
                # to_out + residual -> norm3 -> FeedForward + residual -> proj_out + the block input
                return ops.ff_chain(o, h, x.view(rows, C), self.chain, shape=(n, H, W, C))
            h = ops.linear(o, self.o2, res=h, stats_out=st)
        return self._tail(x, h, st, n, H, W, C)

    def _tail(self, x, h, st, n, H, W, C):
        # GEGLU feed-forward (norm3 folded), proj_out + the block input
        h = _ff(h, st, self.ff1, self.ff2, self.ff2p)
        return ops.conv(h.view(n, H, W, C), self.proj_out, res=x, gn_out=True)


class _Motion:
    def __init__(self, dv, p, c, heads, groups, kw):
        t = p + ".temporal_transformer"
        b = t + ".transformer_blocks.0"
        sd = dv.sd
        self.c, self.heads, self.groups = c, heads, groups
        self.norm = (dv.f32(t + ".norm.weight"), dv.f32(t + ".norm.bias"))
        self.proj_in = dv.packed(t + ".proj_in.weight", t + ".proj_in.bias")
        self.proj_out = dv.packed(t + ".proj_out.weight", t + ".proj_out.bias")
        self.attn = []
        i = 0
        max_len = kw.get("temporal_position_encoding_max_len", 24)
        while f"{b}.attention_blocks.{i}.to_q.weight" in sd:
            a = f"{b}.attention_blocks.{i}"
            pe = sd.get(a + ".pos_encoder.pe")
            if kw.get("temporal_position_encoding", False):
                pe = (pe.reshape(-1, c) if pe is not None else positional_encoding(c, max_len)).float()
                pe = pe.to(dv.device).contiguous()
            else:
                pe = None
            ln = (sd[f"{b}.norms.{i}.weight"], sd[f"{b}.norms.{i}.bias"])
            wqkv = [sd[f"{a}.to_{n}.weight"] for n in "qkv"]
            self.attn.append(dict(
                qkv=dv.packed_ln(torch.cat(wqkv, 0), None, ln, pe=pe),
                # LayerNorm + pe + q|k|v + temporal SDPA in one kernel (ls_temporal_attention)
                fused=ops.pack_temporal(*wqkv, *ln, pe, heads, dv.device) if c in (320, 640) and heads == 8
                else None,
                o=dv.packed(a + ".to_out.0.weight", a + ".to_out.0.bias")))
            i += 1
        self.ff1 = dv.packed_ln(sd[b + ".ff.net.0.proj.weight"], sd[b + ".ff.net.0.proj.bias"],
                                (sd[b + ".ff_norm.weight"], sd[b + ".ff_norm.bias"]), geglu=True)
        self.ff2 = dv.packed(b + ".ff.net.2.weight", b + ".ff.net.2.bias")
        self.ff2p = _ff2_packed(dv, b + ".ff.net.2.weight")
        # the last attention block's to_out + ff_norm + ff + proj_out in one launch (ls_ff_chain)
        self.chain = _chain_pack(self.attn[-1]["o"], self.ff1, self.ff2, self.proj_out, c) if self.attn else None

    def __call__(self, x, B):
        n, H, W, C = x.shape
        F = n // B
        S = H * W
        rows = n * S
        d = C // self.heads
        sc = ops.group_norm(x, self.groups, 1e-6, *self.norm, n)
        lns = torch.empty((rows, 2), dtype=torch.float32, device=x.device)  # LN stats of h, from its GEMM
        # GN affine folded into the row-block GEMM's A rows (32x32 / 16x16); materialised elsewhere
        h = ops.conv(x, self.proj_in, aff=(sc[0], sc[1], 1, False), aff_materialize=True,
                     stats_out=lns).view(rows, C)
        o = torch.empty((rows, C), dtype=torch.bfloat16, device=x.device)
        fuse = _FUSED_TEMPORAL and ops.temporal_attention_ok(C, self.heads, F, S)
        for i, a in enumerate(self.attn):
            if fuse and a["fused"] is not None:
                # LayerNorm (+pe) -> q|k|v -> SDPA over the frames: q|k|v never reach HBM
                ops.temporal_attention(h, a["fused"], B, F, S, out=o)
            else:
                pk = a["qkv"]  # LN (+ positional encoding, as the W pe row table) folded in
                rv = (pk.pe_rows, S, pk.pe_rows.shape[1], F) if pk.pe_rows is not None else None
                qkv = ops.linear(h, pk, ln_stats=lns, rowvec=rv)
                # "(b f) s c -> (b s) f c": batch (b, s), sequence f
                st = (F * S * 3 * C, 3 * C, S * 3 * C, d)
                ops.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=B * S, z2=S, heads=self.heads, nq=F, nk=F,
                              head_dim=d, qs=st, ks=st, vs=st, os_=(F * S * C, C, S * C, d))
            if i == len(self.attn) - 1 and ops.ff_chain_ok(o, self.chain):
                # to_out + residual -> ff_norm -> FeedForward + residual -> proj_out + the module input
                return ops.ff_chain(o, h, x.view(rows, C), self.chain, shape=(n, H, W, C))
            h = ops.linear(o, a["o"], res=h, stats_out=lns)
        h = _ff(h, lns, self.ff1, self.ff2, self.ff2p)
        return ops.conv(h.view(n, H, W, C), self.proj_out, res=x, gn_out=True)


class _DeviceUNet:
    """All packed weights on one device + the forward schedule."""

    def __init__(self, sd, cfg, device):
        dv = _Dev(sd, device)
        self.cfg, self.device = cfg, device
        boc = list(cfg["block_out_channels"])
        nb = len(boc)
        heads = cfg["attention_head_dim"]
        heads = list(heads) if isinstance(heads, (list, tuple)) else [heads] * nb
        groups, eps = cfg["norm_num_groups"], float(cfg["norm_eps"])
        lpb = cfg["layers_per_block"]
        audio = cfg["add_audio_layer"]
        mkw = cfg.get("motion_module_kwargs") or {}
        mheads = mkw.get("num_attention_heads", 8)
        self.cin = cfg["in_channels"]
        self.cin_pad = (self.cin + 7) // 8 * 8
        self.cout = cfg["out_channels"]
        self.boc = boc
        self.temb_dim = boc[0] * 4
        self.flip, self.shift = bool(cfg["flip_sin_to_cos"]), float(cfg["freq_shift"])
        bfw = lambda k: sd[k].to(torch.bfloat16).to(device).contiguous()  # ls_small_linear: plain [N][K]
        self.t1, self.t1b = bfw("time_embedding.linear_1.weight"), dv.f32("time_embedding.linear_1.bias")
        self.t2, self.t2b = bfw("time_embedding.linear_2.weight"), dv.f32("time_embedding.linear_2.bias")
        self.conv_in = dv.packed("conv_in.weight", "conv_in.bias", cin_pad=self.cin_pad)
        temb_w, temb_b = [], []

        def resnet(p, cin, cout, scale=1.0):
            slot = sum(w.shape[0] for w in temb_w)
            temb_w.append(sd[p + ".time_emb_proj.weight"])
            temb_b.append(sd[p + ".time_emb_proj.bias"])
            return _Resnet(dv, p, cin, cout, groups, eps, scale, slot)

        def motion(p, c):
            if f"{p}.temporal_transformer.norm.weight" not in sd:
                return None
            return _Motion(dv, p, c, mheads, groups, mkw)

        self.down = []
        out_c = boc[0]
        for i, bt in enumerate(cfg["down_block_types"]):
            in_c, out_c = out_c, boc[i]
            layers = []
            for l in range(lpb):
                p = f"down_blocks.{i}"
                r = resnet(f"{p}.resnets.{l}", in_c if l == 0 else out_c, out_c)
                a = _Transformer(dv, f"{p}.attentions.{l}", out_c, heads[i], groups, audio) \
                    if bt == "CrossAttnDownBlock3D" else None
                layers.append((r, a, motion(f"{p}.motion_modules.{l}", out_c)))
            ds = dv.packed(f"down_blocks.{i}.downsamplers.0.conv.weight", f"down_blocks.{i}.downsamplers.0.conv.bias") \
                if i < nb - 1 else None
            self.down.append((layers, ds))
        c = boc[-1]
        ms = float(cfg["mid_block_scale_factor"])
        self.mid = (resnet("mid_block.resnets.0", c, c, ms),
                    _Transformer(dv, "mid_block.attentions.0", c, heads[-1], groups, audio),
                    motion("mid_block.motion_modules.0", c),
                    resnet("mid_block.resnets.1", c, c, ms))
        rev = list(reversed(boc))
        rheads = list(reversed(heads))
        self.up = []
        out_c = rev[0]
        for i, bt in enumerate(cfg["up_block_types"]):
            prev_c, out_c = out_c, rev[i]
            in_c = rev[min(i + 1, nb - 1)]
            layers = []
            for l in range(lpb + 1):
                p = f"up_blocks.{i}"
                skip_c = in_c if l == lpb else out_c
                r_in = prev_c if l == 0 else out_c
                r = resnet(f"{p}.resnets.{l}", r_in + skip_c, out_c)
                a = _Transformer(dv, f"{p}.attentions.{l}", out_c, rheads[i], groups, audio) \
                    if bt == "CrossAttnUpBlock3D" else None
                layers.append((r, a, motion(f"{p}.motion_modules.{l}", out_c)))
            us = dv.packed(f"up_blocks.{i}.upsamplers.0.conv.weight", f"up_blocks.{i}.upsamplers.0.conv.bias") \
                if i < nb - 1 else None
            self.up.append((layers, us))
        self.norm_out = (dv.f32("conv_norm_out.weight"), dv.f32("conv_norm_out.bias"))
        self.groups, self.eps = groups, eps
        # 8 output columns (out_channels used): the narrow halo-tile conv (N = 8 / 16) stores 16-B
        # rows and takes conv_norm_out + SiLU in its halo transform
        self.conv_out = dv.packed("conv_out.weight", "conv_out.bias",
                                  n_pad=(self.cout + 7) // 8 * 8 if self.cout <= 16 and _NARROW_OUT else None)
        self.temb_w = torch.cat(temb_w, 0).to(torch.bfloat16).to(device).contiguous()
        self.temb_b = torch.cat(temb_b, 0).float().to(device).contiguous()

    def audio_kv(self, audio_rows):
        """k|v projections of the audio rows for every Transformer3DModel, in forward
        order (down, mid, up) -- constant over the denoising loop."""
        order = [a for layers, _ in self.down for _, a, _ in layers if a is not None] + [self.mid[1]] + \
                [a for layers, _ in self.up for _, a, _ in layers if a is not None]
        return {id(a): a.audio_kv(audio_rows) for a in order}

    def transformers(self):
        for layers, _ in self.down + self.up:
            for _, a, _ in layers:
                if a is not None:
                    yield a
        yield self.mid[1]

    def temb(self, ts_i32, step_i32, B, t_rows=None):
        """The time embedding projected for every resnet.  In the denoising loop every
        sample of the batch has the same timestep (the reference expands one t over the
        batch, unet.py:361-374), so it is ONE row -- the resnets read it as a row vector
        spanning all B samples (computed per sample until round 5: 48 identical rows through
        three GEMVs, 0.8 ms of a 48-window step).  ``t_rows``: fp32 timesteps, one per
        sample (or one for all), from forward()'s float / per-sample timestep argument."""
        if t_rows is not None:
            t = ops.timestep_embed_f32(t_rows, self.boc[0], self.flip, self.shift)
        else:
            t = ops.timestep_embed(ts_i32, step_i32, 1, self.boc[0], self.flip, self.shift)
        e1 = ops.small_linear(t, self.t1, self.t1b)
        emb = ops.small_linear(e1, self.t2, self.t2b, silu_in=True)
        return ops.small_linear(emb, self.temb_w, self.temb_b, silu_in=True)

    def forward(self, x_in, B, ts_i32, step_i32, audio_rows, n_audio_tok, down_res=None, mid_res=None,
                audio_kv=None, t_rows=None):
        """x_in NHWC bf16 (B*F, H, W, cin_pad) -> eps NHWC bf16 (B*F, H, W, n) with out_channels
        used of n (8 for the UNet's 4: conv_out runs on the narrow halo tile).
        audio_kv: the dict of audio_kv(audio_rows), precomputed once per window batch.
        t_rows: fp32 timesteps (1 or B values) instead of ts_i32[step_i32]."""
        kvs = audio_kv or {}
        temb = self.temb(ts_i32, step_i32, B, t_rows)
        h = ops.conv(x_in, self.conv_in, gn_out=True)
        skips = [h]
        for layers, ds in self.down:
            for r, a, m in layers:
                h = r(h, B, temb)
                if a is not None:
                    h = a(h, audio_rows, n_audio_tok, kvs.get(id(a)))
                if m is not None:
                    h = m(h, B)
                skips.append(h)
            if ds is not None:
                h = ops.conv(h, ds, stride=2, pad=1, gn_out=True)
                skips.append(h)
        if down_res is not None:
            skips = [s + r for s, r in zip(skips, down_res)]
        r0, a, m, r1 = self.mid
        h = r0(h, B, temb)
        h = a(h, audio_rows, n_audio_tok, kvs.get(id(a)))
        if m is not None:
            h = m(h, B)
        h = r1(h, B, temb)
        if mid_res is not None:
            h = h + mid_res
        for layers, us in self.up:
            for r, a, m in layers:
                h = r(h, B, temb, x2=skips.pop())
                if a is not None:
                    h = a(h, audio_rows, n_audio_tok, kvs.get(id(a)))
                if m is not None:
                    h = m(h, B)
            if us is not None:
                h = ops.conv(h, us, upsample=True, gn_out=True)
        sc = ops.group_norm(h, self.groups, self.eps, *self.norm_out, B)
        if not _NARROW_OUT:
            return ops.conv(ops.group_norm_apply(h, sc[0], sc[1], B, True), self.conv_out)
        return ops.conv(h, self.conv_out, aff=(sc[0], sc[1], h.shape[0] // B, True), aff_materialize=True)


# --------------------------------------------------------------------------
# public drop-in class
# --------------------------------------------------------------------------


class UNet3DConditionModel(torch.nn.Module):
    """Drop-in for latentsync.models.unet.UNet3DConditionModel (unet.py:39-512)."""

    _supports_gradient_checkpointing = False

    def __init__(self, **kwargs):
        super().__init__()
        unknown = set(kwargs) - set(_DEFAULTS)
        if unknown:
            raise TypeError(f"unexpected UNet3DConditionModel arguments: {sorted(unknown)}")
        cfg = dict(_DEFAULTS)
        cfg.update(kwargs)
        cfg["norm_eps"] = float(cfg["norm_eps"])
        if cfg["mid_block_type"] != "UNetMidBlock3DCrossAttn":
            raise ValueError(f"unknown mid_block_type : {cfg['mid_block_type']}")
        for bt in list(cfg["down_block_types"]) + list(cfg["up_block_types"]):
            bt = bt[7:] if bt.startswith("UNetRes") else bt
            if bt not in ("DownBlock3D", "CrossAttnDownBlock3D", "UpBlock3D", "CrossAttnUpBlock3D"):
                raise ValueError(f"{bt} does not exist.")
        if cfg["dual_cross_attention"]:
            raise NotImplementedError
        if cfg["use_linear_projection"] or cfg["class_embed_type"] or cfg["num_class_embeds"] or \
                cfg["resnet_time_scale_shift"] != "default" or cfg["use_inflated_groupnorm"]:
            raise NotImplementedError("configuration outside the LatentSync inference path")
        self._internal_dict = FrozenDict(cfg)
        self.sample_size = cfg["sample_size"]
        self.use_motion_module = cfg["use_motion_module"]
        self.add_audio_layer = cfg["add_audio_layer"]
        self._shapes = unet_param_shapes(cfg)
        # reference __init__ draws nn defaults; weights here come from the
        # deterministic generator (seed 0, drawn lazily) until a checkpoint is
        # loaded or init_weights(seed) is called.
        self._sd_store = None
        self._device = torch.device("cpu")
        self._dev = None
        self.num_upsamplers = len(cfg["block_out_channels"]) - 1

    # -- config / attributes the pipeline reads ----------------------------
    @property
    def config(self):
        return self._internal_dict

    @property
    def dtype(self):
        return torch.bfloat16

    @property
    def device(self):
        return self._device

    @classmethod
    def from_config(cls, config):
        return cls(**dict(config))

    def set_attention_precision(self, precision):
        """'bf16' (default; the reference's SDPA at bf16) or 'fp8': the spatial
        self attention (sequences > 128 tokens) computes P V on the block-scaled e4m3
        MFMA (ls_attention_fp8) -- BASELINE.json configs[4].  Not a reference API."""
        if precision not in ("bf16", "fp8"):
            raise ValueError(f"attention precision {precision!r}: 'bf16' or 'fp8'")
        self._attn_fp8 = precision == "fp8"
        if self._dev is not None:
            for a in self._dev.transformers():
                a.fp8 = self._attn_fp8

    def set_attention_slice(self, slice_size):
        """Accepted for API compatibility (unet.py:243-306); the flash kernel never
        materialises the attention matrix, so slicing is a no-op."""
        return None

    # -- weights ------------------------------------------------------------
    @property
    def _sd(self):
        if self._sd_store is None:
            self._sd_store = {}
            self.init_weights(0, _pack=False)
        return self._sd_store

    def state_dict(self, *a, **k):
        return dict(self._sd)

    def load_state_dict(self, state_dict, strict=True):
        """unet.py:473-492 drop rules, then strict/non-strict key matching."""
        state_dict = dict(state_dict)
        if "conv_in.weight" in state_dict and state_dict["conv_in.weight"].shape[1] != self.config.in_channels:
            del state_dict["conv_in.weight"]
            state_dict.pop("conv_in.bias", None)
        if "conv_out.weight" in state_dict and state_dict["conv_out.weight"].shape[0] != self.config.out_channels:
            del state_dict["conv_out.weight"]
            state_dict.pop("conv_out.bias", None)
        for key in [k for k in state_dict if "attn2.to_k." in k or "attn2.to_v." in k]:
            if state_dict[key].shape[1] != self.config.cross_attention_dim:
                del state_dict[key]
        missing = [k for k in self._shapes if k not in state_dict]
        unexpected = [k for k in state_dict if k not in self._shapes]
        if strict and (missing or unexpected):
            raise RuntimeError(f"Error(s) in loading state_dict: missing {missing[:5]}, unexpected {unexpected[:5]}")
        for k, v in state_dict.items():
            if k in self._shapes:
                if tuple(v.shape) != tuple(self._shapes[k]):
                    raise RuntimeError(f"size mismatch for {k}: {tuple(v.shape)} vs {self._shapes[k]}")
                self._sd[k] = v.detach().float().cpu()
        self._dev = None
        if self._device.type == "cuda":
            self._pack()
        return missing, unexpected

    @classmethod
    def from_pretrained(cls, model_config: dict, ckpt_path: str, device="cpu"):
        """unet.py:494-512: (unet, resume_global_step)."""
        unet = cls.from_config(model_config)
        step = 0
        if ckpt_path != "":
            ckpt = torch.load(ckpt_path, map_location="cpu", weights_only=True)
            step = ckpt.get("global_step", 0)
            unet.load_state_dict(ckpt["state_dict"], strict=False)
        return unet.to(device), step

    def init_weights(self, seed: int, _pack=True):
        """Deterministic reference-independent weights (latentsync_amd.weights)."""
        sd = fill_state_dict(self._shapes, seed)
        for k in self._shapes:
            if k.endswith("pos_encoder.pe"):
                sd[k] = positional_encoding(self._shapes[k][-1], self._shapes[k][1])[None]
        self._sd_store = sd
        self._dev = None
        if _pack and self._device.type == "cuda":
            self._pack()
        return self

    def _pack(self):
        self._dev = _DeviceUNet(self._sd, self.config, self._device)
        for a in self._dev.transformers():
            a.fp8 = getattr(self, "_attn_fp8", False)

    def to(self, device=None, dtype=None, *a, **k):
        if isinstance(device, torch.dtype):
            device, dtype = None, device
        if device is not None:
            device = torch.device(device)
            if device.type == "cuda" and device.index is None:
                device = torch.device("cuda", torch.cuda.current_device())
            if device != self._device:
                self._device = device
                self._dev = None
                if device.type == "cuda":
                    self._pack()
        return self

    def cuda(self, device=None):
        return self.to(torch.device("cuda", device) if device is not None else "cuda")

    def train(self, mode=True):
        if mode:
            raise NotImplementedError("training is out of scope (SURVEY.md §2)")
        self.training = False
        return self

    def eval(self):
        self.training = False
        return self

    # -- forward -------------------------------------------------------------
    def _require_device(self):
        if self._dev is None:
            raise RuntimeError("UNet3DConditionModel runs only on the MI355X HIP path: call .to('cuda') first")
        return self._dev

    def forward(self, sample, timestep, encoder_hidden_states=None, class_labels=None, attention_mask=None,
                down_block_additional_residuals=None, mid_block_additional_residual=None, return_dict=True):
        """unet.py:312-471.  ``attention_mask`` is accepted and, as in the reference
        (whose down/up blocks never forward it to the attention), has no effect."""
        dev = self._require_device()
        B, Cin, F, H, W = sample.shape
        if Cin != self.config.in_channels:
            raise ValueError(f"expected {self.config.in_channels} input channels, got {Cin}")
        if H % (2 ** self.num_upsamplers) or W % (2 ** self.num_upsamplers):
            raise NotImplementedError("sample size must be a multiple of the overall up-sampling factor")
        if self.config.center_input_sample:
            sample = 2 * sample - 1.0
        x = torch.zeros((B * F, H, W, dev.cin_pad), dtype=torch.bfloat16, device=sample.device)
        x[..., :Cin] = sample.permute(0, 2, 3, 4, 1).reshape(B * F, H, W, Cin)
        # time (unet.py:361-376): a python int / float or a tensor of one value or one per
        # sample, broadcast over the batch; get_timestep_embedding takes it as fp32
        if torch.is_tensor(timestep):
            tv = timestep.reshape(-1)
            if tv.numel() not in (1, B):
                raise ValueError(f"timestep has {tv.numel()} values for a batch of {B}")
        else:
            tv = torch.tensor([float(timestep)], dtype=torch.float64)
        tv = tv.to(sample.device).to(torch.float32)
        if tv.numel() > 1 and bool((tv == tv[0]).all()):
            tv = tv[:1]  # one row spans the batch (the denoising loop's case)
        ts = step = None
        audio, ntok = None, 0
        if encoder_hidden_states is not None and self.add_audio_layer:
            ehs = encoder_hidden_states
            if ehs.dim() == 4:
                ehs = ehs.reshape(-1, ehs.shape[-2], ehs.shape[-1])
            ntok = ehs.shape[1]
            audio = ehs.to(torch.bfloat16).reshape(-1, ehs.shape[-1]).contiguous()
        dres = None
        if down_block_additional_residuals is not None:
            dres = []
            for r in down_block_additional_residuals:
                if r.dim() == 4:
                    r = r.unsqueeze(2)
                rb, rc, rf, rh, rw = r.shape
                dres.append(r.expand(B, rc, F, rh, rw).permute(0, 2, 3, 4, 1).reshape(B * F, rh, rw, rc)
                            .to(torch.bfloat16))
        mres = None
        if mid_block_additional_residual is not None:
            r = mid_block_additional_residual
            if r.dim() == 4:
                r = r.unsqueeze(2)
            rb, rc, rf, rh, rw = r.shape
            mres = r.expand(B, rc, F, rh, rw).permute(0, 2, 3, 4, 1).reshape(B * F, rh, rw, rc).to(torch.bfloat16)
        eps = dev.forward(x, B, ts, step, audio, ntok, dres, mres, t_rows=tv.contiguous())
        out = eps.reshape(B, F, H, W, -1)[..., :self.config.out_channels].permute(0, 4, 1, 2, 3)
        out = out.to(sample.dtype if sample.dtype.is_floating_point else torch.float32).contiguous()
        if not return_dict:
            return (out,)
        return UNet3DConditionOutput(sample=out)

    __call__ = torch.nn.Module.__call__
