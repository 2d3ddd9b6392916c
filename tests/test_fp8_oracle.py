"""CPU checks of the fp8 attention restatement (oracle/fp8_cpu.py): the MX block
quantisation of V and the fp8 attention emulation against fp32 SDPA, at the
tolerance tests/test_gpu_fp8.py states for the GPU kernel."""
import math

import torch
import torch.nn.functional as F

from conftest import rel_err
from oracle import fp8_cpu as Q


def test_key_perm_is_a_permutation():
    assert sorted(Q.key_perm().tolist()) == list(range(128))


def test_quant_vt_round_trip_and_scale_range():
    g = torch.Generator().manual_seed(0)
    nk, D = 300, 40
    mag = torch.pow(2.0, torch.randint(-20, 20, (nk, 1), generator=g).float())
    v = (torch.randn(nk, D, generator=g) * mag).to(torch.bfloat16).float()
    v[5:9] = 0.0  # zero rows inside a tile
    v[256:] = 0.0  # an all-zero tile: scale 2^-127
    codes, e8 = Q.quant_vt(v)
    assert codes.shape == (3, D, 128) and e8.shape == (3, D, 4)
    vq = Q.dequant_vt(codes, e8, nk)
    # the row max of a tile lands in [128, 256) before rounding (256 after, at worst): never near 448
    vals = codes.view(torch.float8_e4m3fn).float().view(3, D, 128).abs().amax(-1)
    nz = vals > 0
    assert bool(((vals[nz] >= 128) & (vals[nz] <= 256)).all())
    # e4m3 round to nearest: |err| <= 2^-4 |v| for normal codes, <= half a subnormal step below
    step = torch.pow(2.0, e8.double() - 127 - 9).float()  # e4m3 subnormal spacing 2^-9, scaled
    blk_step = torch.empty(3, D, 128)
    blk_step[:, :, Q.key_perm()] = step.repeat_interleave(32, -1)
    blk_step = blk_step.permute(0, 2, 1).reshape(-1, D)[:nk]
    assert bool(((vq - v).abs() <= torch.maximum(v.abs() / 16, blk_step / 2) + 1e-30).all())


def test_attention_emulation_within_stated_tolerance():
    g = torch.Generator().manual_seed(1)
    nq, nk, D = 256, 700, 40
    q = torch.randn(nq, D, generator=g).to(torch.bfloat16).float() * 2
    k = torch.randn(nk, D, generator=g).to(torch.bfloat16).float()
    v = torch.randn(nk, D, generator=g).to(torch.bfloat16).float()
    o = Q.attention_fp8(q, k, v, 1 / math.sqrt(D))
    ref = F.scaled_dot_product_attention(q[None], k[None], v[None])[0]
    assert rel_err(o, ref) < 6e-2
