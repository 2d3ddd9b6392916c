"""SD AutoencoderKL (stabilityai/sd-vae-ft-mse architecture) on the HIP path --
the ``vae`` object LipsyncPipeline calls (lipsync_pipeline.py:145-149, 296, 315).

diffusers 0.32.2 is not part of the reference tree and not installed; this is a
restatement of its published algorithm (parity against
the CPU oracle, "parity unpinned" against diffusers itself).  Same public surface
as diffusers: ``encode(x).latent_dist.sample(generator)``, ``decode(z).sample``,
``config.scaling_factor / shift_factor / block_out_channels / latent_channels``,
``enable_slicing`` / ``disable_slicing``.  Internally NHWC bf16.  GroupNorm:
statistics from the producing conv's epilogue column sums (ops.conv(gn_out=True)
-> ls_groupnorm_colsum, no read pass), the affine (+SiLU) materialised once by
ls_groupnorm_apply -- a 3x3 conv's gather would recompute it for each of its 9
taps.  Mid attention on the flash kernel (1 head, d = 512).
"""
import os
from dataclasses import dataclass

import torch

from . import ops
from .schema import vae_param_shapes
from .unet import _Dev, FrozenDict
from .weights import fill_state_dict


class _MutableConfig(dict):
    """diffusers configs are attribute-accessible; the reference assigns
    ``vae.config.scaling_factor`` / ``shift_factor`` (scripts/inference.py:57-58)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


class _Res:
    def __init__(self, dv, p):
        self.n1 = (dv.f32(p + ".norm1.weight"), dv.f32(p + ".norm1.bias"))
        self.n2 = (dv.f32(p + ".norm2.weight"), dv.f32(p + ".norm2.bias"))
        self.c1 = dv.packed(p + ".conv1.weight", p + ".conv1.bias")
        self.c2 = dv.packed(p + ".conv2.weight", p + ".conv2.bias")
        self.sc = dv.packed(p + ".conv_shortcut.weight", p + ".conv_shortcut.bias") \
            if (p + ".conv_shortcut.weight") in dv.sd else None

    def __call__(self, x):
        n = x.shape[0]
        s1 = ops.group_norm(x, 32, 1e-6, *self.n1, n)
        # GN affine + SiLU fused into the halo-tile 3x3 conv where it takes the call, else
        # materialised once (ops.conv aff_materialize)
        h = ops.conv(x, self.c1, aff=(s1[0], s1[1], 1, True), aff_materialize=True, gn_out=True)
        s2 = ops.group_norm(h, 32, 1e-6, *self.n2, n)
        res = x if self.sc is None else ops.conv(x, self.sc)
        return ops.conv(h, self.c2, aff=(s2[0], s2[1], 1, True), aff_materialize=True, res=res, gn_out=True)


class _Attn:
    def __init__(self, dv, p):
        sd = dv.sd
        self.gn = (dv.f32(p + ".group_norm.weight"), dv.f32(p + ".group_norm.bias"))
        self.qkv = dv.packed(None, w=torch.cat([sd[p + f".to_{n}.weight"] for n in "qkv"], 0),
                             b=torch.cat([sd[p + f".to_{n}.bias"] for n in "qkv"], 0))
        self.out = dv.packed(p + ".to_out.0.weight", p + ".to_out.0.bias")

    def __call__(self, x):
        n, H, W, C = x.shape
        N = H * W
        s = ops.group_norm(x, 32, 1e-6, *self.gn, n)
        qkv = ops.conv(ops.group_norm_apply(x, s[0], s[1], n, False), self.qkv).view(n * N, 3 * C)
        o = torch.empty((n * N, C), dtype=torch.bfloat16, device=x.device)
        st = (N * 3 * C, 0, 3 * C, C)
        ops.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=n, z2=1, heads=1, nq=N, nk=N, head_dim=C, qs=st,
                      ks=st, vs=st, os_=(N * C, 0, C, C))
        return ops.conv(o.view(n, H, W, C), self.out, res=x, gn_out=True)


class _DeviceVAE:
    def __init__(self, sd, boc, lpb, latent, device):
        dv = _Dev(sd, device)
        self.boc, self.lpb, self.latent = boc, lpb, latent
        self.enc_in = dv.packed("encoder.conv_in.weight", "encoder.conv_in.bias", cin_pad=8)
        self.enc = []
        for i in range(len(boc)):
            res = [_Res(dv, f"encoder.down_blocks.{i}.resnets.{l}") for l in range(lpb)]
            ds = dv.packed(f"encoder.down_blocks.{i}.downsamplers.0.conv.weight",
                           f"encoder.down_blocks.{i}.downsamplers.0.conv.bias") if i < len(boc) - 1 else None
            self.enc.append((res, ds))
        self.enc_mid = (_Res(dv, "encoder.mid_block.resnets.0"), _Attn(dv, "encoder.mid_block.attentions.0"),
                        _Res(dv, "encoder.mid_block.resnets.1"))
        self.enc_norm = (dv.f32("encoder.conv_norm_out.weight"), dv.f32("encoder.conv_norm_out.bias"))
        self.enc_out = dv.packed("encoder.conv_out.weight", "encoder.conv_out.bias")
        self.quant = dv.packed("quant_conv.weight", "quant_conv.bias")
        self.post_quant = dv.packed("post_quant_conv.weight", "post_quant_conv.bias", cin_pad=8, n_pad=8)
        self.dec_in = dv.packed("decoder.conv_in.weight", "decoder.conv_in.bias", cin_pad=8)
        self.dec_mid = (_Res(dv, "decoder.mid_block.resnets.0"), _Attn(dv, "decoder.mid_block.attentions.0"),
                        _Res(dv, "decoder.mid_block.resnets.1"))
        self.dec = []
        for i in range(len(boc)):
            res = [_Res(dv, f"decoder.up_blocks.{i}.resnets.{l}") for l in range(lpb + 1)]
            us = dv.packed(f"decoder.up_blocks.{i}.upsamplers.0.conv.weight",
                           f"decoder.up_blocks.{i}.upsamplers.0.conv.bias") if i < len(boc) - 1 else None
            self.dec.append((res, us))
        self.dec_norm = (dv.f32("decoder.conv_norm_out.weight"), dv.f32("decoder.conv_norm_out.bias"))
        # 8 output columns (3 used): the narrow halo-tile conv stores 16-B rows
        self.dec_out = dv.packed("decoder.conv_out.weight", "decoder.conv_out.bias", n_pad=8)

    def encode_moments(self, x):
        """x NHWC bf16 (n, R, R, 8) (3 used channels) -> moments fp32 (n, R/8, R/8, 8)."""
        h = ops.conv(x, self.enc_in, gn_out=True)
        for res, ds in self.enc:
            for r in res:
                h = r(h)
            if ds is not None:
                H = h.shape[1]
                h = ops.conv(h, ds, stride=2, pad=0, out_hw=(H // 2, h.shape[2] // 2),  # F.pad(0,1,0,1) + s2
                             gn_out=True)
        for blk in self.enc_mid:
            h = blk(h)
        s = ops.group_norm(h, 32, 1e-6, *self.enc_norm, h.shape[0])
        # conv_norm_out + SiLU fused into conv_out's halo transform (the narrow halo tile)
        h = ops.conv(h, self.enc_out, aff=(s[0], s[1], 1, True), aff_materialize=True)
        return ops.conv(h, self.quant, out_f32=True)

    def decode(self, z):
        """z NHWC bf16 (n, h, w, 8) (4 used channels, already / scaling) -> (n, 8h, 8w, 8) bf16
        (3 used channels)."""
        h = ops.conv(z, self.post_quant)
        h = ops.conv(h, self.dec_in, gn_out=True)
        for blk in self.dec_mid:
            h = blk(h)
        for res, us in self.dec:
            for r in res:
                h = r(h)
            if us is not None:
                h = ops.conv(h, us, upsample=True, gn_out=True)
        s = ops.group_norm(h, 32, 1e-6, *self.dec_norm, h.shape[0])
        return ops.conv(h, self.dec_out, aff=(s[0], s[1], 1, True), aff_materialize=True)


class DiagonalGaussianDistribution:
    """diffusers DiagonalGaussianDistribution over NCHW moments."""

    def __init__(self, moments):
        self.parameters = moments
        self.mean, logvar = torch.chunk(moments, 2, dim=1)
        self.logvar = torch.clamp(logvar, -30.0, 20.0)
        self.std = torch.exp(0.5 * self.logvar)
        self.var = torch.exp(self.logvar)

    def sample(self, generator=None):
        eps = torch.randn(self.mean.shape, generator=generator, device=self.mean.device, dtype=self.mean.dtype)
        return self.mean + self.std * eps

    def mode(self):
        return self.mean


@dataclass
class AutoencoderKLOutput:
    latent_dist: DiagonalGaussianDistribution


@dataclass
class DecoderOutput:
    sample: torch.Tensor


class AutoencoderKL(torch.nn.Module):
    def __init__(self, in_channels=3, out_channels=3, block_out_channels=(128, 256, 512, 512), layers_per_block=2,
                 latent_channels=4, norm_num_groups=32, sample_size=512, scaling_factor=0.18215, shift_factor=None,
                 **kw):
        super().__init__()
        if in_channels != 3 or out_channels != 3 or norm_num_groups != 32:
            raise NotImplementedError("only the SD AutoencoderKL layout is on the LatentSync path")
        object.__setattr__(self, "_cfg", _MutableConfig(
            in_channels=in_channels, out_channels=out_channels, block_out_channels=list(block_out_channels),
            layers_per_block=layers_per_block, latent_channels=latent_channels, norm_num_groups=norm_num_groups,
            sample_size=sample_size, scaling_factor=scaling_factor, shift_factor=shift_factor))
        self._shapes = vae_param_shapes(tuple(block_out_channels), layers_per_block, latent_channels)
        self._sd = None  # drawn lazily (seed 0) unless loaded / init_weights(seed)
        self._device = torch.device("cpu")
        self._dev = None
        self.use_slicing = False

    @property
    def config(self):
        return self._cfg

    @property
    def dtype(self):
        return torch.bfloat16

    @property
    def device(self):
        return self._device

    # legacy diffusers mid-attention names (query/key/value/proj_attn)
    _LEGACY = {".query.": ".to_q.", ".key.": ".to_k.", ".value.": ".to_v.", ".proj_attn.": ".to_out.0."}

    def load_state_dict(self, state_dict, strict=True):
        sd = {}
        for k, v in state_dict.items():
            for a, b in self._LEGACY.items():
                if "attentions" in k and a in k:
                    k = k.replace(a, b)
            if v.dim() == 4 and "attentions" in k and v.shape[-1] == 1:  # legacy 1x1-conv attn weights
                v = v[:, :, 0, 0]
            sd[k] = v
        missing = [k for k in self._shapes if k not in sd]
        unexpected = [k for k in sd if k not in self._shapes]
        if strict and (missing or unexpected):
            raise RuntimeError(f"AutoencoderKL state_dict mismatch: missing {missing[:5]}, unexpected {unexpected[:5]}")
        if self._sd is None:
            self._sd = fill_state_dict(self._shapes, 0)
        for k, v in sd.items():
            if k in self._shapes:
                self._sd[k] = v.detach().float().cpu()
        self._dev = None
        if self._device.type == "cuda":
            self._pack()
        return missing, unexpected

    @classmethod
    def from_pretrained(cls, path, subfolder=None, **kw):
        """Local diffusers directory (config.json + diffusion_pytorch_model.safetensors)."""
        import json
        d = os.path.join(path, subfolder) if subfolder else path
        if not os.path.isdir(d):
            raise RuntimeError(f"AutoencoderKL.from_pretrained: {path!r} is not a local directory "
                               "(no network access: hub names cannot be fetched)")
        cfg = {}
        if os.path.exists(os.path.join(d, "config.json")):
            with open(os.path.join(d, "config.json")) as f:
                cfg = {k: v for k, v in json.load(f).items() if not k.startswith("_")}
        vae = cls(**cfg)
        from safetensors.torch import load_file
        st = os.path.join(d, "diffusion_pytorch_model.safetensors")
        if os.path.exists(st):
            vae.load_state_dict(load_file(st))
        else:
            vae.load_state_dict(torch.load(os.path.join(d, "diffusion_pytorch_model.bin"), map_location="cpu",
                                           weights_only=True))
        return vae

    def init_weights(self, seed):
        self._sd = fill_state_dict(self._shapes, seed)
        self._dev = None
        if self._device.type == "cuda":
            self._pack()
        return self

    def _pack(self):
        if self._sd is None:
            self._sd = fill_state_dict(self._shapes, 0)
        c = self._cfg
        self._dev = _DeviceVAE(self._sd, c.block_out_channels, c.layers_per_block, c.latent_channels, self._device)

    def to(self, device=None, dtype=None, *a, **k):
        if isinstance(device, torch.dtype):
            device = None
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

    def enable_slicing(self):
        self.use_slicing = True

    def disable_slicing(self):
        self.use_slicing = False

    def _require(self):
        if self._dev is None:
            raise RuntimeError("AutoencoderKL runs only on the MI355X HIP path: call .to('cuda') first")
        return self._dev

    def encode(self, x, return_dict=True):
        dev = self._require()
        n, c, H, W = x.shape
        xin = torch.zeros((n, H, W, 8), dtype=torch.bfloat16, device=x.device)
        xin[..., :c] = x.permute(0, 2, 3, 1)
        mom = dev.encode_moments(xin).permute(0, 3, 1, 2).contiguous()
        post = DiagonalGaussianDistribution(mom.to(x.dtype if x.dtype.is_floating_point else torch.float32))
        return AutoencoderKLOutput(latent_dist=post) if return_dict else (post,)

    def decode(self, z, return_dict=True, generator=None):
        dev = self._require()
        n, c, h, w = z.shape
        zin = torch.zeros((n, h, w, 8), dtype=torch.bfloat16, device=z.device)
        zin[..., :c] = z.permute(0, 2, 3, 1)
        out = dev.decode(zin)[..., :3].permute(0, 3, 1, 2).to(z.dtype).contiguous()
        return DecoderOutput(sample=out) if return_dict else (out,)
