"""The fused temporal attention (ls_temporal_attention, latentsync_amd/csrc/ls_motion.hip)
on MI355X: LayerNorm + positional encoding + q|k|v + SDPA over the frames of every
pixel (motion_module.py:203-218, :262-313) against a plain PyTorch fp32 reference of the
same op on the same bf16-rounded inputs, and the whole motion module (fused path)
against the fp32 oracle (oracle/ref_cpu.py motion_module, pinned to the reference's
golden at C = 64) and against the unfused q|k|v GEMM + ls_attention path.

Tolerance: rel-L2 2e-2 (bf16 LayerNorm output, bf16 q/k/v, bf16 P, bf16 o; as the
other attention tests)."""
import math
from collections import OrderedDict

import pytest
import torch
import torch.nn.functional as F

from conftest import block_sd, rel_err
from latentsync_amd import ops, schema as S
from latentsync_amd import unet as U

pytestmark = pytest.mark.gpu


def _ref(x, wq, wk, wv, gamma, beta, pe, B, Fr, Sp, heads):
    """The reference block in fp32: x rows (b f) s, C."""
    C = x.shape[1]
    n = F.layer_norm(x, (C,), gamma, beta, 1e-5)
    n = n.reshape(B, Fr, Sp, C).permute(0, 2, 1, 3).reshape(B * Sp, Fr, C)  # (b f) s c -> (b s) f c
    if pe is not None:
        n = n + pe[:Fr]
    q, k, v = n @ wq.T, n @ wk.T, n @ wv.T
    sp = lambda t: t.reshape(B * Sp, Fr, heads, C // heads).permute(0, 2, 1, 3)
    o = F.scaled_dot_product_attention(sp(q), sp(k), sp(v))
    o = o.permute(0, 2, 1, 3).reshape(B, Sp, Fr, C).permute(0, 2, 1, 3).reshape(B * Fr * Sp, C)
    return o


@pytest.mark.parametrize("C,B,Fr,Sp", [(320, 2, 16, 32), (320, 1, 5, 16), (640, 3, 16, 16), (640, 1, 7, 8),
                                       (320, 1, 16, 1024)])
def test_temporal_attention_kernel(gpu, C, B, Fr, Sp):
    g = torch.Generator().manual_seed(C + Fr)
    heads = 8
    x = (torch.randn((B * Fr * Sp, C), generator=g) * 2 + 0.5).to(torch.bfloat16).float()
    wq, wk, wv = (torch.randn((C, C), generator=g) / math.sqrt(C) for _ in range(3))
    gamma = 1 + 0.1 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    pe = U.positional_encoding(C, 24)
    pk = ops.pack_temporal(wq, wk, wv, gamma, beta, pe, heads, gpu)
    # the reference on the kernel's bf16 weights (q unscaled back), fp32 math
    wb = pk.w.float().cpu()
    sc = math.log2(math.e) / math.sqrt(C // heads)
    tiles = wb.reshape(C // 16, 3, 16, C)  # (q_t, k_t, v_t) per 16-channel tile, in channel order
    wq_b, wk_b, wv_b = (tiles[:, k].reshape(C, C) for k in range(3))
    wq_b = wq_b / sc
    ref = _ref(x, wq_b, wk_b, wv_b, gamma, beta, pe, B, Fr, Sp, heads)
    out = ops.temporal_attention(x.to(torch.bfloat16).to(gpu), pk, B, Fr, Sp).float().cpu()
    e = rel_err(out, ref)
    print(f"ls_temporal_attention C={C} B={B} F={Fr} S={Sp}: rel_err {e:.5f}")
    assert e < 2e-2
    # every row written, nothing past them
    assert torch.isfinite(out).all()


def test_temporal_attention_rejects_bad_shapes(gpu):
    C = 320
    pk = ops.pack_temporal(*(torch.zeros(C, C) for _ in range(3)), torch.ones(C), torch.zeros(C), None, 8, gpu)
    x = torch.zeros((17 * 8, C), dtype=torch.bfloat16, device=gpu)
    with pytest.raises(RuntimeError, match="F <= 16"):
        ops.temporal_attention(x, pk, 1, 17, 8)
    assert not ops.temporal_attention_ok(320, 8, 16, 8) and ops.temporal_attention_ok(640, 8, 16, 8)


def _shapes(fn, *a):
    sd = OrderedDict()
    fn(sd, "blk", *a)
    return OrderedDict((k[4:], v) for k, v in sd.items())


@pytest.mark.parametrize("C,Hh", [(320, 4), (640, 4)])
def test_motion_module_fused(gpu, C, Hh, monkeypatch):
    """The whole VanillaTemporalModule with the fused attention, at the UNet's own
    widths (32x32 / 16x16 levels), against the fp32 oracle and the unfused path."""
    from latentsync_amd.config import STAGE2_MODEL
    from oracle import ref_cpu as R
    kw = STAGE2_MODEL["motion_module_kwargs"]
    sd = block_sd("blk", _shapes(S._motion, C, kw), 17)  # pe buffers: the sinusoid default on both sides
    m = U._Motion(U._Dev(sd, torch.device("cuda")), "blk", C, 8, 32, kw)
    assert all(a["fused"] is not None for a in m.attn)
    g = torch.Generator().manual_seed(C)
    B, Fr = 2, 16
    x = torch.randn((B, C, Fr, Hh, Hh), generator=g).to(torch.bfloat16).float()
    xd = x.permute(0, 2, 3, 4, 1).reshape(B * Fr, Hh, Hh, C).to(torch.bfloat16).cuda().contiguous()
    y = m(xd, B).float().cpu()
    monkeypatch.setattr(U, "_FUSED_TEMPORAL", False)
    y0 = m(xd, B).float().cpu()
    ref = R.motion_module(x, sd, "blk", 8, 32)
    yr = y.reshape(B, Fr, Hh, Hh, C).permute(0, 4, 1, 2, 3)
    e, e0 = rel_err(yr, ref), rel_err(y0.reshape(B, Fr, Hh, Hh, C).permute(0, 4, 1, 2, 3), ref)
    print(f"motion module C={C}: fused vs oracle {e:.5f}, unfused vs oracle {e0:.5f}")
    assert e < 2e-2 and e0 < 2e-2
    assert rel_err(y, y0) < 2e-2

