"""Deterministic, reference-independent weight generator.

No checkpoint of the reference is available offline, so every
parity fixture and every benchmark uses weights drawn from this generator.  Each
tensor is a pure function of (state_dict key, shape, base seed), so the golden
generator (which overwrites the *reference* modules' parameters), the CPU oracle
and the HIP path all see bit-identical fp32 weights.

Rules:
  * ``*.weight`` with ndim >= 2   -> N(0,1) / sqrt(fan_in)        (Linear / conv)
  * 1-D ``*.weight``             -> 1 + 0.1 * N(0,1)               (GroupNorm / LayerNorm gain)
  * ``*.bias``                   -> 0.05 * N(0,1)
The reference zero-initialises ``conv_in``, ``conv_out`` and every motion-module
``proj_out`` (latentsync/models/unet.py:92,241; motion_module.py:65-66).  With
zeros the UNet output is identically 0, so this generator deliberately
re-randomises them like any other weight.  Buffers (``pos_encoder.pe``,
``positional_embedding``) are computed, never drawn.
"""
import math
import zlib

import torch

_BUFFER_SUFFIXES = ("pos_encoder.pe", "positional_embedding")


def key_seed(key: str, base_seed: int = 0) -> int:
    return (zlib.crc32(key.encode("utf-8")) ^ ((base_seed * 0x9E3779B1) & 0xFFFFFFFF)) & 0xFFFFFFFF


def init_tensor(key: str, shape, base_seed: int = 0) -> torch.Tensor:
    shape = tuple(int(s) for s in shape)
    g = torch.Generator().manual_seed(key_seed(key, base_seed))
    t = torch.randn(shape, generator=g, dtype=torch.float32)
    if key.endswith(".bias"):
        return t.mul_(0.05)
    if len(shape) >= 2:
        fan_in = 1
        for s in shape[1:]:
            fan_in *= s
        return t.mul_(1.0 / math.sqrt(fan_in))
    return t.mul_(0.1).add_(1.0)


def is_buffer_key(key: str) -> bool:
    return key.endswith(_BUFFER_SUFFIXES)


def fill_state_dict(shapes: dict, base_seed: int = 0) -> dict:
    """shapes: {key: shape}. Returns {key: fp32 tensor} for every non-buffer key."""
    return {k: init_tensor(k, s, base_seed) for k, s in shapes.items() if not is_buffer_key(k)}


def randomize_module_(module: torch.nn.Module, base_seed: int = 0) -> None:
    """Overwrite every parameter of an nn.Module in place (used on the reference
    modules by oracle/make_golden.py)."""
    with torch.no_grad():
        for k, p in module.named_parameters():
            p.copy_(init_tensor(k, p.shape, base_seed).to(p.dtype))
