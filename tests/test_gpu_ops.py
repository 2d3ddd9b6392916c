"""Per-kernel parity on MI355X: every C-ABI entry point against a plain
PyTorch fp32 CPU reference of the same op, on the same bf16-rounded inputs.
Tolerances are stated per test (bf16 output rounding + fp32 accumulation)."""
import ctypes
import math

import pytest
import torch
import torch.nn.functional as F

from conftest import rel_err
from latentsync_amd import ops
from latentsync_amd.packing import geglu_interleave, pack_weight, pad_bias

pytestmark = pytest.mark.gpu
DEV = "cuda"


def bf(t):
    return t.to(torch.bfloat16).float()


def rnd(*shape, seed=0, scale=1.0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)) * scale


def packed(w, b, ksize, cin_pad=None, geglu=False, n_pad=None):
    n_out = w.shape[0]
    if geglu:
        w, b = geglu_interleave(w, b)
    wp = pack_weight(w, cin_pad=cin_pad, n_pad=n_pad)
    bp = pad_bias(b, n_pad)
    cin = cin_pad or (w.shape[1] + 7) // 8 * 8
    return ops.Packed(wp.to(torch.bfloat16).to(DEV), None if bp is None else bp.to(DEV), cin, ksize, n_out, geglu)


def nhwc(x):  # (n, C, H, W) -> (n, H, W, C) bf16 device
    return x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(DEV)


def nchw(y):
    return y.float().cpu().permute(0, 3, 1, 2)


@pytest.mark.parametrize("cin,cout,stride,up,split", [(64, 96, 1, False, 0), (64, 64, 2, False, 0),
                                                      (16, 320, 1, False, 0), (128, 64, 1, True, 0),
                                                      (640, 1280, 1, False, 4), (8, 40, 1, False, 0)])
def test_conv3x3(gpu, cin, cout, stride, up, split):
    n, H = 3, 8
    x = bf(rnd(n, cin, H, H, seed=1))
    w = bf(rnd(cout, cin, 3, 3, seed=2, scale=1 / math.sqrt(9 * cin)))
    b = rnd(cout, seed=3, scale=0.1)
    xin = F.interpolate(x, scale_factor=2.0, mode="nearest") if up else x
    ref = F.conv2d(xin, w, b, stride=stride, padding=1)
    y = ops.conv(nhwc(x), packed(w, b, 3), stride=stride, upsample=up, split_k=split)
    assert rel_err(nchw(y), ref) < 1e-2


def test_conv3x3_vae_downsample(gpu):
    x = bf(rnd(2, 64, 8, 8, seed=4))
    w = bf(rnd(64, 64, 3, 3, seed=5, scale=1 / 24))
    b = rnd(64, seed=6, scale=0.1)
    ref = F.conv2d(F.pad(x, (0, 1, 0, 1)), w, b, stride=2)
    y = ops.conv(nhwc(x), packed(w, b, 3), stride=2, pad=0, out_hw=(4, 4))
    assert rel_err(nchw(y), ref) < 1e-2


def test_conv_groupnorm_silu_temb_residual_concat(gpu):
    """ResnetBlock3D conv1/conv2 fusion: GN5D(+SiLU) prologue, temb + residual
    epilogue, concat (x, skip) gather."""
    B, Fr, H, c1, c2, cout, groups = 2, 4, 8, 64, 32, 64, 32
    x1 = bf(rnd(B * Fr, c1, H, H, seed=7))
    x2 = bf(rnd(B * Fr, c2, H, H, seed=8))
    xc = torch.cat([x1, x2], 1)
    gamma, beta = 1 + 0.1 * rnd(c1 + c2, seed=9), 0.1 * rnd(c1 + c2, seed=10)
    w = bf(rnd(cout, c1 + c2, 3, 3, seed=11, scale=1 / math.sqrt(9 * (c1 + c2))))
    b = rnd(cout, seed=12, scale=0.1)
    temb = rnd(B, cout, seed=13)
    res = bf(rnd(B * Fr, cout, H, H, seed=14))
    x5 = xc.reshape(B, Fr, c1 + c2, H, H).permute(0, 2, 1, 3, 4)
    g5 = F.silu(F.group_norm(x5, groups, gamma, beta, 1e-5))
    g4 = g5.permute(0, 2, 1, 3, 4).reshape(B * Fr, c1 + c2, H, H)
    ref = F.conv2d(g4, w, b, padding=1) + temb.repeat_interleave(Fr, 0)[:, :, None, None]
    ref = (ref + res) * 0.5
    sc, sh = ops.group_norm(nhwc(x1), groups, 1e-5, gamma.to(DEV), beta.to(DEV), B, x2=nhwc(x2))
    y = ops.conv(nhwc(x1), packed(w, b, 3), x2=nhwc(x2), aff=(sc, sh, Fr, True),
                 rowvec=(temb.to(DEV), Fr * H * H, cout), res=nhwc(res), out_scale=0.5)
    assert rel_err(nchw(y), ref) < 1e-2


@pytest.mark.parametrize("C,groups,spp", [(320, 32, 16), (2560, 32, 1), (128, 32, 1), (96, 32, 4)])
def test_groupnorm_stats(gpu, C, groups, spp):
    n, H = 16, 4
    x = bf(rnd(n, C, H, H, seed=20) * 3 + 5)  # large mean: exercises the shifted sums
    gamma, beta = 1 + 0.1 * rnd(C, seed=21), 0.1 * rnd(C, seed=22)
    S = n // spp
    sc, sh = ops.group_norm(nhwc(x), groups, 1e-6, gamma.to(DEV), beta.to(DEV), S)
    y = ops.affine_act(nhwc(x), sc, sh, S, False)
    x5 = x.reshape(S, spp, C, H, H).permute(0, 2, 1, 3, 4)
    ref = F.group_norm(x5, groups, gamma, beta, 1e-6).permute(0, 2, 1, 3, 4).reshape(n, C, H, H)
    assert rel_err(nchw(y), ref) < 1e-2


@pytest.mark.parametrize("M,K,N,act,split", [(200, 320, 960, 0, 0), (256, 1280, 10240, 1, 0),
                                              (100, 384, 640, 0, 0), (256, 5120, 1280, 0, 3),
                                              (64, 640, 5120, 1, 2), (300, 384, 1536, 2, 0)])
def test_linear(gpu, M, K, N, act, split):
    x = bf(rnd(M, K, seed=30))
    w = bf(rnd(N, K, seed=31, scale=1 / math.sqrt(K)))
    b = rnd(N, seed=32, scale=0.1)
    res = bf(rnd(M, N // 2 if act == 1 else N, seed=33))
    y_ref = x @ w.T + b
    if act == ops.ACT_GEGLU:
        h, g = y_ref.chunk(2, -1)
        ref = h * F.gelu(g)
        y = ops.linear(x.to(torch.bfloat16).to(DEV), packed(w, b, 1, geglu=True), act=act, split_k=split)
    elif act == ops.ACT_GELU:
        ref = F.gelu(y_ref)
        y = ops.linear(x.to(torch.bfloat16).to(DEV), packed(w, b, 1), act=act, split_k=split)
    else:
        ref = y_ref + res
        y = ops.linear(x.to(torch.bfloat16).to(DEV), packed(w, b, 1), res=res.to(torch.bfloat16).to(DEV),
                       split_k=split)
    assert rel_err(y.float().cpu(), ref) < 1e-2


def test_linear_fp32_out(gpu):
    x = bf(rnd(64, 512, seed=34))
    w = bf(rnd(8, 512, seed=35, scale=1 / 16))
    y = ops.linear(x.to(torch.bfloat16).to(DEV), packed(w, None, 1), out_f32=True)
    assert y.dtype == torch.float32
    assert rel_err(y.cpu(), x @ w.T) < 1e-5


@pytest.mark.parametrize("C", [320, 1280, 384])
def test_layernorm_pe(gpu, C):
    rows, S, Fr = 4 * 16 * 2, 4, 16
    x = bf(rnd(rows, C, seed=40) * 2 + 1)
    g, b = 1 + 0.1 * rnd(C, seed=41), 0.1 * rnd(C, seed=42)
    pe = rnd(24, C, seed=43)
    ref = F.layer_norm(x, (C,), g, b, 1e-5)
    f = (torch.arange(rows) // S) % Fr
    ref = ref + pe[f]
    y = ops.layer_norm(x.to(torch.bfloat16).to(DEV), g.to(DEV), b.to(DEV), 1e-5, pe=pe.to(DEV),
                       pe_rows_per_frame=S, pe_frames=Fr)
    assert rel_err(y.float().cpu(), ref) < 1e-2


def _sdpa(q, k, v, scale=None):
    return F.scaled_dot_product_attention(q, k, v, scale=scale)


@pytest.mark.parametrize("n,N,Nk,heads,d", [(4, 256, 256, 8, 40), (2, 64, 64, 8, 80), (2, 16, 16, 8, 160),
                                            (3, 256, 50, 8, 40), (2, 64, 50, 8, 160), (1, 100, 100, 6, 64),
                                            (2, 64, 64, 1, 512), (2, 1024, 1024, 1, 128), (2, 64, 64, 8, 4),
                                            (2, 1000, 777, 8, 40), (2, 200, 130, 8, 80),
                                            # configs[4] (latent 64^2): spatial N = 4096 / 1024, audio cross
                                            (1, 4096, 4096, 8, 40), (2, 1024, 1024, 8, 80), (1, 4096, 50, 8, 40),
                                            # SD-VAE mid attention at 256^2: 1 head, d = 512, N = 1024
                                            (2, 1024, 1024, 1, 512),
                                            # d = 512 (attnw): ragged queries / keys, two heads
                                            (2, 300, 130, 2, 512)])
def test_attention_spatial(gpu, n, N, Nk, heads, d):
    C = heads * d
    q = bf(rnd(n, N, C, seed=50))
    k = bf(rnd(n, Nk, C, seed=51))
    v = bf(rnd(n, Nk, C, seed=52))
    split = lambda t: t.reshape(t.shape[0], t.shape[1], heads, d).permute(0, 2, 1, 3)
    ref = _sdpa(split(q), split(k), split(v)).permute(0, 2, 1, 3).reshape(n, N, C)
    qd, kd, vd = (t.to(torch.bfloat16).to(DEV) for t in (q, k, v))
    o = torch.empty_like(qd)
    ops.attention(qd, kd, vd, o, batch=n, z2=1, heads=heads, nq=N, nk=Nk, head_dim=d, qs=(N * C, 0, C, d),
                  ks=(Nk * C, 0, C, d), vs=(Nk * C, 0, C, d), os_=(N * C, 0, C, d))
    assert rel_err(o.float().cpu(), ref) < 1.5e-2


@pytest.mark.parametrize("qscale", [1.0, 3.0])
def test_attention_d512_rescale(gpu, qscale):
    """attnw (d = 512): keys whose scores grow along the sequence, so the running max moves
    past the lazy-rescale threshold on later tiles (qscale 3: log2-unit logits past 20)."""
    n, N, Nk, d = 2, 256, 1024, 512
    q = rnd(n, N, d, seed=60) * qscale
    k = rnd(n, Nk, d, seed=61) * torch.linspace(0.2, 2.0, Nk).reshape(1, Nk, 1)
    v = rnd(n, Nk, d, seed=62)
    q, k, v = bf(q), bf(k), bf(v)
    ref = _sdpa(q[:, None], k[:, None], v[:, None])[:, 0]
    qd, kd, vd = (t.to(torch.bfloat16).to(DEV) for t in (q, k, v))
    o = torch.empty_like(qd)
    ops.attention(qd, kd, vd, o, batch=n, z2=1, heads=1, nq=N, nk=Nk, head_dim=d, qs=(N * d, 0, d, d),
                  ks=(Nk * d, 0, d, d), vs=(Nk * d, 0, d, d), os_=(N * d, 0, d, d))
    assert rel_err(o.float().cpu(), ref) < 1.5e-2


@pytest.mark.parametrize("n_img,L,hw", [(2, 50, 1024), (3, 64, 256), (1, 7, 128)])
def test_cross_attention_block(gpu, n_img, L, hw):
    """ls_cross_attention_block (norm2 + to_q + SDPA over the audio tokens + to_out +
    residual, one launch; attention.py:174-199) against fp32: y and the row statistics
    of the stored y rows."""
    C, H, D = 320, 8, 40
    M = n_img * hw
    g = torch.Generator().manual_seed(80 + L)
    r = lambda *s, sc=1.0: torch.randn(*s, generator=g) * sc
    x = bf(r(M, C) * 1.5 + 0.3)
    gamma, beta = 1 + 0.1 * r(C), 0.1 * r(C)
    wq, wo, bo = r(C, C, sc=C ** -0.5), r(C, C, sc=C ** -0.5), 0.1 * r(C)
    kv = bf(r(n_img * L, 2 * C))
    xd, kvd = x.to(torch.bfloat16).to(DEV), kv.to(torch.bfloat16).to(DEV)
    st = ops.row_stats(xd)
    pk = ops.pack_cross_attention(wq, gamma, beta, wo, bo, H, DEV)
    st2 = torch.empty_like(st)
    assert ops.cross_attention_ok(xd, pk, L, hw)
    y = ops.cross_attention_block(xd, st, pk, kvd, L, hw, st2).float().cpu()
    ln = torch.nn.functional.layer_norm(x, (C,), gamma, beta, eps=1e-5)
    q = (ln @ wq.T).reshape(n_img, hw, H, D).permute(0, 2, 1, 3)
    k = kv[:, :C].reshape(n_img, L, H, D).permute(0, 2, 1, 3)
    v = kv[:, C:].reshape(n_img, L, H, D).permute(0, 2, 1, 3)
    o = _sdpa(q, k, v).permute(0, 2, 1, 3).reshape(M, C)
    ref = o @ wo.T + bo + x
    e = rel_err(y, ref)
    print("cross-attention block rel_err", n_img, L, hw, e)
    assert e < 1.5e-2
    # the (mean, rstd) of the stored bf16 y rows (norm3's fold)
    mean, var = y.double().mean(1), y.double().var(1, unbiased=False)
    s2 = st2.cpu().double()
    assert torch.allclose(s2[:, 0], mean, rtol=1e-4, atol=1e-4)
    assert torch.allclose(s2[:, 1], 1 / torch.sqrt(var + 1e-5), rtol=1e-4)


@pytest.mark.parametrize("kernel", ["attn5", "attn6"])
@pytest.mark.parametrize("qscale,N,Nk", [(1.0, 1024, 1024), (3.0, 1024, 1024), (3.0, 777, 1000)])
def test_attention_d40_rescale_fused_qkv(gpu, qscale, N, Nk, kernel):
    """The d = 40 self-attention kernel (attn6, 32x32x16 MFMA) on the UNet's fused q|k|v
    rows (row stride 3C) with keys whose scores grow along the sequence, so the running
    max moves past the lazy-rescale threshold on later tiles (qscale 3: log2-unit logits
    past 20); ragged query / key counts in the last case."""
    n, heads, d = 2, 8, 40
    C = heads * d
    q = rnd(n, N, C, seed=70) * qscale
    k = rnd(n, Nk, C, seed=71) * torch.linspace(0.2, 2.0, Nk).reshape(1, Nk, 1)
    v = rnd(n, Nk, C, seed=72)
    q, k, v = bf(q), bf(k), bf(v)
    split = lambda t: t.reshape(t.shape[0], t.shape[1], heads, d).permute(0, 2, 1, 3)
    ref = _sdpa(split(q), split(k), split(v)).permute(0, 2, 1, 3).reshape(n, N, C)
    L = max(N, Nk)
    qkv = torch.zeros((n, L, 3 * C), dtype=torch.bfloat16)
    qkv[:, :N, :C], qkv[:, :Nk, C:2 * C], qkv[:, :Nk, 2 * C:] = q.to(torch.bfloat16), k.to(torch.bfloat16), \
        v.to(torch.bfloat16)
    qkv = qkv.to(DEV).reshape(n * L, 3 * C)
    o = torch.empty((n * N, C), dtype=torch.bfloat16, device=DEV)
    st = (L * 3 * C, 0, 3 * C, d)
    from latentsync_amd import _lib
    if _lib.load().ls_set_tuning(9, int(kernel == "attn6")) != 0:  # the 32x32x16 kernel (A/B option) or attn5
        pytest.skip("attn6 is compiled only in the diagnostics build (LS_DIAG_BUILD=1)")
    try:
        ops.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=n, z2=1, heads=heads, nq=N, nk=Nk, head_dim=d,
                      qs=st, ks=st, vs=st, os_=(N * C, 0, C, d))
    finally:
        _lib.load().ls_set_tuning(9, 0)
    assert rel_err(o.float().cpu().reshape(n, N, C), ref) < 1.5e-2


@pytest.mark.parametrize("C,Fr,S", [(320, 16, 16), (640, 16, 16), (1280, 16, 16), (320, 12, 15), (640, 7, 9),
                                    (1280, 16, 3)])
def test_attention_temporal_strided(gpu, C, Fr, S):
    """VersatileAttention: '(b f) s c -> (b s) f c' read straight from the fused
    q|k|v rows (motion_module.py:265, 300) -- the short-sequence kernel, incl.
    fewer frames than 16 and (pixel) batches that do not fill its blocks."""
    B, heads = 2, 8
    d = C // heads
    qkv = bf(rnd(B * Fr * S, 3 * C, seed=60))
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    re = lambda t: t.reshape(B, Fr, S, C).permute(0, 2, 1, 3).reshape(B * S, Fr, heads, d).permute(0, 2, 1, 3)
    o_ref = _sdpa(re(q), re(k), re(v)).permute(0, 2, 1, 3).reshape(B, S, Fr, C).permute(0, 2, 1, 3).reshape(-1, C)
    qd = qkv.to(torch.bfloat16).to(DEV)
    o = torch.empty((B * Fr * S, C), dtype=torch.bfloat16, device=DEV)
    st = (Fr * S * 3 * C, 3 * C, S * 3 * C, d)
    ops.attention(qd, qd[:, C:], qd[:, 2 * C:], o, batch=B * S, z2=S, heads=heads, nq=Fr, nk=Fr, head_dim=d, qs=st,
                  ks=st, vs=st, os_=(Fr * S * C, C, S * C, d))
    assert rel_err(o.float().cpu(), o_ref) < 1.5e-2


@pytest.mark.parametrize("M", [2, 8, 19])
def test_small_linear_and_timestep(gpu, M):
    from oracle import ref_cpu as R
    x = rnd(M, 1280, seed=70)
    w = bf(rnd(3000, 1280, seed=71, scale=1 / 36))
    b = rnd(3000, seed=72)
    y = ops.small_linear(x.to(DEV), w.to(torch.bfloat16).to(DEV), b.to(DEV), silu_in=True)
    assert rel_err(y.cpu(), F.silu(x) @ w.T + b) < 1e-5
    ts = torch.tensor([951, 501, 1], dtype=torch.int32, device=DEV)
    for i, t in enumerate((951, 501, 1)):
        step = torch.tensor([i], dtype=torch.int32, device=DEV)
        e = ops.timestep_embed(ts, step, 2, 320, True, 0.0)
        ref = R.timestep_embedding(torch.tensor([t, t]), 320, True, 0)
        assert (e.cpu() - ref).abs().max() < 2e-3  # sin/cos of args up to ~951 rad in fp32


def test_ddim_cfg_step(gpu):
    from oracle import ref_cpu as R
    P, g = 4 * 8 * 8, 1.5
    ac = R.ddim_alphas_cumprod()
    ts = R.ddim_timesteps(20)
    coef = []
    for t in ts:
        prev = t - 1000 // 20
        a_t = ac[t]
        a_p = ac[prev] if prev >= 0 else ac[0]
        coef.append([a_t.sqrt(), (1 - a_t).sqrt(), a_p.sqrt(), (1 - a_p).sqrt()])
    coef = torch.tensor(coef, dtype=torch.float32).to(DEV)
    lat = rnd(P, 4, seed=80)
    eps = bf(rnd(2 * P, 4, seed=81))
    step = torch.tensor([3], dtype=torch.int32, device=DEV)
    unet_in = torch.zeros((2 * P, 16), dtype=torch.bfloat16, device=DEV)
    latd = lat.clone().to(DEV)
    ops.ddim_cfg_step(eps.to(torch.bfloat16).to(DEV), 2, g, latd, coef, step, unet_in)
    u, a = eps[:P], eps[P:]
    ref = R.ddim_step(ac, u + g * (a - u), int(ts[3]), lat, 20)
    assert rel_err(latd.cpu(), ref) < 1e-5
    assert int(step.item()) == 4
    assert rel_err(unet_in[:P, :4].float().cpu(), ref) < 1e-2
    assert rel_err(unet_in[P:, :4].float().cpu(), ref) < 1e-2


@pytest.fixture
def forced_tile():
    from latentsync_amd import _lib
    lib = _lib.load()

    def force(tile, split=0):
        if lib.ls_set_tuning(2, tile) != 0:  # tile ids 7 / 8: diagnostics build only
            pytest.skip(f"tile {tile} is compiled only in the diagnostics build (LS_DIAG_BUILD=1)")
        lib.ls_set_tuning(3, split)
    yield force
    lib.ls_set_tuning(2, 0)
    lib.ls_set_tuning(3, 0)


@pytest.mark.parametrize("tile", [1, 2, 3, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("case", ["linear_res", "geglu", "conv3x3", "conv3x3_up_s2", "split2"])
def test_gemm_tiles(gpu, forced_tile, tile, case):
    """Every tile configuration of ls_conv2d (incl. the 8-wave 256-row kernel) on
    ragged M / N, fused epilogues and TAPU 3x3 gathers.  Tolerance 1e-2 (bf16 out)."""
    if case in ("linear_res", "geglu", "split2"):
        M, K, N = 700, 640, (1024 if case == "geglu" else 320)
        act = ops.ACT_GEGLU if case == "geglu" else 0
        x = bf(rnd(M, K, seed=40))
        w = bf(rnd(N, K, seed=41, scale=1 / math.sqrt(K)))
        b = rnd(N, seed=42, scale=0.1)
        forced_tile(tile, 2 if case == "split2" else 0)
        if act:
            h, g = (x @ w.T + b).chunk(2, -1)
            ref = h * F.gelu(g)
            y = ops.linear(x.to(torch.bfloat16).to(DEV), packed(w, b, 1, geglu=True), act=act)
        else:
            res = bf(rnd(M, N, seed=43))
            ref = x @ w.T + b + res
            y = ops.linear(x.to(torch.bfloat16).to(DEV), packed(w, b, 1), res=res.to(torch.bfloat16).to(DEV))
        assert rel_err(y.float().cpu(), ref) < 1e-2
    else:
        up = case == "conv3x3_up_s2"
        n, H, cin, cout = 5, 12, 128, 192
        x = bf(rnd(n, cin, H, H, seed=44))
        w = bf(rnd(cout, cin, 3, 3, seed=45, scale=1 / math.sqrt(9 * cin)))
        b = rnd(cout, seed=46, scale=0.1)
        forced_tile(tile)
        if up:
            ref = F.conv2d(F.interpolate(x, scale_factor=2.0, mode="nearest"), w, b, padding=1)
            y = ops.conv(nhwc(x), packed(w, b, 3), upsample=True)
            assert rel_err(nchw(y), ref) < 1e-2
            ref = F.conv2d(x, w, b, stride=2, padding=1)
            y = ops.conv(nhwc(x), packed(w, b, 3), stride=2)
        else:
            ref = F.conv2d(x, w, b, padding=1)
            y = ops.conv(nhwc(x), packed(w, b, 3))
        assert rel_err(nchw(y), ref) < 1e-2


def test_linear_strided_views(gpu):
    """Row-strided input / residual / output views (the Whisper stacked-layer layout)."""
    M, C = 300, 384
    X = bf(rnd(M, 3, C, seed=47)).to(torch.bfloat16).to(DEV)
    w = bf(rnd(C, C, seed=48, scale=1 / math.sqrt(C)))
    b = rnd(C, seed=49, scale=0.1)
    ops.linear(X[:, 0], packed(w, b, 1), res=X[:, 1], out=X[:, 2])
    Xc = X.float().cpu()
    ref = Xc[:, 0] @ w.T + b + Xc[:, 1]
    assert rel_err(Xc[:, 2], ref) < 1e-2
    ln = ops.layer_norm(X[:, 1], torch.ones(C, device=DEV), torch.zeros(C, device=DEV))
    assert rel_err(ln.float().cpu(), F.layer_norm(Xc[:, 1], (C,))) < 1e-2


@pytest.mark.parametrize("geglu,pe", [(False, False), (True, False), (False, True)])
def test_layernorm_folded_linear(gpu, geglu, pe):
    """LayerNorm -> linear folded into the GEMM epilogue (ls_row_stats +
    ln_rowstats/ln_colsum, + W pe row table with modulo) vs F.layer_norm then
    linear in fp32.  Rows carry a large mean to exercise the (acc - mean*colsum)
    cancellation.  Tolerance 1e-2."""
    from latentsync_amd.unet import _Dev
    M, C, N, S, Fr = 512, 320, (1280 if geglu else 960), 16, 8
    x = bf(rnd(M, C, seed=80) * 2 + 3)
    gamma, beta = 1 + 0.1 * rnd(C, seed=81), 0.1 * rnd(C, seed=82)
    w = rnd(N, C, seed=83, scale=1 / math.sqrt(C))
    b = rnd(N, seed=84, scale=0.1) if geglu else None
    pe_t = rnd(24, C, seed=85) if pe else None
    t = F.layer_norm(x, (C,), gamma, beta, 1e-5)
    if pe:
        t = t + pe_t[(torch.arange(M) // S) % Fr]
    y_ref = t @ w.T + (b if b is not None else 0)
    pk = _Dev({}, DEV).packed_ln(w, b, (gamma, beta), geglu=geglu, pe=pe_t)
    xd = x.to(torch.bfloat16).to(DEV)
    st = ops.row_stats(xd)
    rv = (pk.pe_rows, S, pk.pe_rows.shape[1], Fr) if pe else None
    if geglu:
        h, g = y_ref.chunk(2, -1)
        y_ref = h * F.gelu(g)
        y = ops.linear(xd, pk, act=ops.ACT_GEGLU, ln_stats=st)
    else:
        y = ops.linear(xd, pk, ln_stats=st, rowvec=rv)
    assert rel_err(y.float().cpu(), y_ref) < 1e-2


@pytest.mark.parametrize("K,M,N,case", [(320, 512, 960, "bias"), (320, 65536, 320, "res"),
                                        (320, 4096, 320, "nobias_res_scale"), (320, 65536, 1024, "geglu"),
                                        (320, 8192, 2560, "ln_geglu"), (320, 65536, 960, "ln_rv"),
                                        (640, 384, 1920, "ln"), (640, 32768, 640, "bias"), (640, 4096, 5120, "ln_geglu"),
                                        (640, 16384, 1920, "ln_rv")])
def test_rowblock_gemm(gpu, K, M, N, case):
    """The row-block short-K kernel (K = 320 / 640, A rows in registers, transposed MFMA,
    register epilogue) for every epilogue flag combination, on N-split grids (small M)
    and the full chunk loop (odd / even chunk counts) -- checked against fp32 on the
    first and last 256 rows, and against the tiled kernel (rowblock off) on all rows.
    Tolerance 1e-2 (bf16 out)."""
    from latentsync_amd import _lib
    lib = _lib.load()
    S, Fr = (1024 if K == 320 else 256), 16
    x = bf(rnd(M, K, seed=90) * (2 if "ln" in case else 1) + (3 if "ln" in case else 0))
    geglu = "geglu" in case
    w = rnd(N, K, seed=91, scale=1 / math.sqrt(K))
    b = None if "nobias" in case else rnd(N, seed=92, scale=0.1)
    xd = x.to(torch.bfloat16).to(DEV)
    kw, scale = {}, 1.0
    rows = torch.cat([torch.arange(256), torch.arange(M - 256, M)])
    if "ln" in case:
        from latentsync_amd.unet import _Dev
        gamma, beta = 1 + 0.1 * rnd(K, seed=93), 0.1 * rnd(K, seed=94)
        pe_t = rnd(24, K, seed=95) if "rv" in case else None
        pk = _Dev({}, DEV).packed_ln(w, b, (gamma, beta), geglu=geglu, pe=pe_t)
        kw["ln_stats"] = ops.row_stats(xd)
        t = F.layer_norm(x[rows], (K,), gamma, beta, 1e-5)
        if pe_t is not None:
            kw["rowvec"] = (pk.pe_rows, S, pk.pe_rows.shape[1], Fr)
            t = t + pe_t[(rows // S) % Fr]
    else:
        pk = packed(w, b, 1, geglu=geglu)
        t = x[rows]
    ref = t @ w.T + (b if b is not None else 0)
    if "res" in case:
        res = bf(rnd(M, N, seed=96))
        kw["res"] = res.to(torch.bfloat16).to(DEV)
        ref = ref + res[rows]
    if "scale" in case:
        scale = 0.5
        ref = ref * scale
    if geglu:
        h, g = ref.chunk(2, -1)
        ref = h * F.gelu(g)
        kw["act"] = ops.ACT_GEGLU
    y = ops.linear(xd, pk, out_scale=scale, **kw)
    lib.ls_set_tuning(6, 0)
    try:
        y_tiled = ops.linear(xd, pk, out_scale=scale, **kw)
    finally:
        lib.ls_set_tuning(6, 1)
    assert rel_err(y.float().cpu()[rows], ref) < 1e-2
    assert rel_err(y.float(), y_tiled.float()) < 1e-2


@pytest.mark.parametrize("M", [512, 65536])
def test_rowblock_uncompiled_flags_fall_back(gpu, M):
    """A row-block-eligible shape (K = 320, 1x1) whose epilogue flags have no compiled
    row-block instance (residual + row vector) must run on the tiled kernels with the
    tiled grid, not the row-block grid (rowblock_flags overwrote ntm/ntn)."""
    K, N, rpv = 320, 320, 256
    x = bf(rnd(M, K, seed=97))
    w = rnd(N, K, seed=98, scale=1 / math.sqrt(K))
    b = rnd(N, seed=99, scale=0.1)
    rv = rnd(M // rpv, N, seed=100)
    res = bf(rnd(M, N, seed=101))
    y = ops.linear(x.to(torch.bfloat16).to(DEV), packed(w, b, 1), res=res.to(torch.bfloat16).to(DEV),
                   rowvec=(rv.to(DEV), rpv, N))
    ref = x @ bf(w).T + b + rv.repeat_interleave(rpv, 0) + res
    assert rel_err(y.float().cpu(), ref) < 1e-2


@pytest.mark.parametrize("K,M,N,res", [(320, 65536, 320, True), (320, 8192, 320, False), (640, 4096, 640, False),
                                       (640, 4096, 640, True), (1280, 2048, 1280, True), (320, 512, 320, True)])
def test_linear_row_stats_out(gpu, K, M, N, res):
    """LayerNorm row statistics of a linear's output emitted with it (row-block epilogue
    when one block owns whole rows, else a trailing ls_row_stats): equal to row_stats()
    of the stored output.  Tolerance 1e-4 (mean) / 1e-3 (rstd)."""
    x = bf(rnd(M, K, seed=97)).to(torch.bfloat16).to(DEV)
    w = rnd(N, K, seed=98, scale=1 / math.sqrt(K))
    b = rnd(N, seed=99, scale=0.5) + 2.0  # rows with |mean| > std
    kw = {"res": bf(rnd(M, N, seed=100)).to(torch.bfloat16).to(DEV)} if res else {}
    st = torch.empty((M, 2), dtype=torch.float32, device=DEV)
    y = ops.linear(x, packed(w, b, 1), stats_out=st, **kw)
    ref = ops.row_stats(y)
    assert (st[:, 0] - ref[:, 0]).abs().max().item() < 1e-4 * max(1.0, ref[:, 0].abs().max().item())
    assert ((st[:, 1] - ref[:, 1]).abs() / ref[:, 1]).max().item() < 1e-3


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("case", ["conv3x3_res", "linear_split2", "rowblock_res"])
def test_gn_colsum(gpu, forced_tile, tile, case):
    """GroupNorm statistics from the producer (ls_conv_desc.gn_colsum_out): the tile
    epilogues and the read-pass fallbacks (small tiles, split-K, row-block) against
    the fp64 sums of the stored bf16 output, and ls_groupnorm_colsum against the
    read-pass ls_groupnorm on the same tensor (fp64 merge: rel 1e-4)."""
    if case == "conv3x3_res":
        n, H, cin, cout, spp = 8, 16, 128, 192, 4
        x = nhwc(bf(rnd(n, cin, H, H, seed=60)))
        pw = packed(bf(rnd(cout, cin, 3, 3, seed=61, scale=1 / math.sqrt(9 * cin))), rnd(cout, seed=62) + 3.0, 3)
        res = nhwc(bf(rnd(n, cout, H, H, seed=63)))
        forced_tile(tile)
        y = ops.conv(x, pw, res=res, gn_out=True)
    else:
        M, K, N = (1024, 640, 320) if case == "linear_split2" else (512, 320, 320)
        n, H, spp, cout = M // 64, 8, 4, N
        x = bf(rnd(M, K, seed=64)).to(torch.bfloat16).to(DEV).view(n, H, H, K)
        pw = packed(bf(rnd(N, K, seed=65, scale=1 / math.sqrt(K))), rnd(N, seed=66) - 2.0, 1)
        res = bf(rnd(M, N, seed=67)).to(torch.bfloat16).to(DEV).view(n, H, H, N)
        forced_tile(tile, 2 if case == "linear_split2" else 0)
        y = ops.conv(x, pw, res=res, gn_out=True, split_k=2 if case == "linear_split2" else 0)
    forced_tile(0)
    cs = y.gn_cs.cpu().double()
    yf = y.float().cpu().double().reshape(-1, 128, cout)
    s1, s2 = yf.sum(1), (yf * yf).sum(1)
    assert (cs[:, 0] - s1).abs().max() <= 1e-5 * yf.abs().sum(1).max()
    assert (cs[:, 1] - s2).abs().max() <= 1e-5 * s2.max()
    S = n // spp
    gamma, beta = (1 + 0.1 * rnd(cout, seed=68)).to(DEV), (0.1 * rnd(cout, seed=69)).to(DEV)
    sc, sh = ops.group_norm(y, 32, 1e-6, gamma, beta, S)
    y2 = y.clone()  # no producer sums: the read pass
    sc2, sh2 = ops.group_norm(y2, 32, 1e-6, gamma, beta, S)
    assert rel_err(sc.cpu(), sc2.cpu()) < 1e-4 and rel_err(sh.cpu(), sh2.cpu()) < 1e-4


def test_groupnorm_colsum_concat(gpu):
    """Up-block GroupNorm over cat(x, skip): both halves' producer sums, groups
    straddling the concat boundary (C1 = 96, C2 = 64, 32 groups of 5)."""
    n, H = 4, 16
    xa = nhwc(bf(rnd(n, 96, H, H, seed=70) * 2 + 1))
    xb = nhwc(bf(rnd(n, 64, H, H, seed=71) - 4))
    ops.gn_colsum(xa)
    ops.gn_colsum(xb)
    gamma, beta = (1 + 0.1 * rnd(160, seed=72)).to(DEV), (0.1 * rnd(160, seed=73)).to(DEV)
    sc, sh = ops.group_norm(xa, 32, 1e-6, gamma, beta, 2, x2=xb)
    sc2, sh2 = ops.group_norm(xa.clone(), 32, 1e-6, gamma, beta, 2, x2=xb.clone())
    assert rel_err(sc.cpu(), sc2.cpu()) < 1e-4 and rel_err(sh.cpu(), sh2.cpu()) < 1e-4


@pytest.mark.parametrize("offset", [10.0, 30.0])
def test_groupnorm_colsum_large_mean(gpu, offset):
    """Column-sum statistics are raw fp32 slot sums (var = E[x^2] - mean^2 in fp64), so
    their relative variance error is ~sqrt(128) eps32 (1 + mean^2 / var) -- here with
    mean / std = 10 and 30 (VAE-decoder-like DC offsets) against the shifted read pass
    and an fp64 reference: scale within 1e-3 (bf16 rounding of y is 3.9e-3)."""
    n, H, C = 8, 32, 128
    x = nhwc(bf(rnd(n, C, H, H, seed=74) + offset))
    ops.gn_colsum(x)
    gamma, beta = (1 + 0.1 * rnd(C, seed=75)).to(DEV), (0.1 * rnd(C, seed=76)).to(DEV)
    sc, sh = ops.group_norm(x, 32, 1e-6, gamma, beta, 2)
    sc2, sh2 = ops.group_norm(x.clone(), 32, 1e-6, gamma, beta, 2)
    xd = x.double().cpu().reshape(2, -1, 32, C // 32)
    var = xd.var(dim=(1, 3), unbiased=False)  # (sample, group)
    ref = gamma.double().cpu().reshape(1, 32, -1) / (var + 1e-6).sqrt()[..., None]
    assert rel_err(sc.cpu().double(), ref.reshape(2, C)) < 1e-3
    assert rel_err(sc.cpu(), sc2.cpu()) < 1e-3 and rel_err(sh.cpu(), sh2.cpu()) < 1e-3


@pytest.mark.parametrize("n,S,H,C1,C2,silu", [(32, 16, 8, 320, 0, True), (24, 8, 4, 1280, 0, True),
                                               (16, 16, 16, 640, 640, True), (6, 1, 32, 128, 0, False),
                                               (16, 4, 2, 2560, 0, True), (5, 1, 3, 64, 32, False)])
def test_groupnorm_apply(gpu, n, S, H, C1, C2, silu):
    """ls_groupnorm_apply: y = act(x * scale[sample, c] + shift[sample, c]) over a channel
    concat, samples of S images (block ranges crossing sample boundaries, ragged tails,
    channel counts split over blockIdx.y), against the same arithmetic in fp32."""
    C = C1 + C2
    x1 = bf(rnd(n, H, H, C1, seed=70))
    x2 = bf(rnd(n, H, H, C2, seed=71)) if C2 else None
    ns = n // S
    sc = rnd(ns, C, seed=72, scale=0.5) + 1.0
    sh = rnd(ns, C, seed=73, scale=0.5)
    y = ops.group_norm_apply(x1.to(torch.bfloat16).to(DEV), sc.to(DEV), sh.to(DEV), ns, silu,
                             x2=x2.to(torch.bfloat16).to(DEV) if C2 else None).float().cpu()
    xx = torch.cat([x1, x2], -1) if C2 else x1
    ref = xx.reshape(ns, S, H, H, C) * sc.reshape(ns, 1, 1, 1, C) + sh.reshape(ns, 1, 1, 1, C)
    ref = (F.silu(ref) if silu else ref).reshape(n, H, H, C)
    err = (y - ref).abs() / (ref.abs() + 1e-2)
    assert float(err.max()) < 1e-2


@pytest.mark.parametrize("K,M,N,H,silu", [(320, 65536, 320, 32, False), (640, 32768, 640, 16, False),
                                          (320, 65536, 960, 32, True), (1280, 512, 1280, 16, False)])
def test_gn_affine_fold(gpu, K, M, N, H, silu):
    """GroupNorm affine (+SiLU) prologue folded into the row-block GEMM's register-resident
    A rows (ls_conv_path 1 for K = 320 / 640; K = 1280 takes the materialising fallback),
    against materialise-then-GEMM; with the LayerNorm row statistics of the output
    (whole rows per block: M >= 256 row blocks, as at the UNet's 32x32 / 16x16 levels)."""
    from latentsync_amd import _lib
    n = M // (H * H)  # per-frame GroupNorm: one sample per image
    x = bf(rnd(M, K, seed=80) * 2 + 1).to(torch.bfloat16).to(DEV).view(n, H, H, K)
    pw = packed(bf(rnd(N, K, seed=81, scale=1 / math.sqrt(K))), rnd(N, seed=82, scale=0.1), 1)
    sc = (1 + 0.2 * rnd(n, K, seed=83)).to(DEV)
    sh = (0.3 * rnd(n, K, seed=84)).to(DEV)
    st1 = torch.empty((M, 2), dtype=torch.float32, device=DEV)
    st2 = torch.empty_like(st1)
    y1 = ops.conv(x, pw, aff=(sc, sh, 1, silu), aff_materialize=True, stats_out=st1)
    y2 = ops.conv(ops.group_norm_apply(x, sc, sh, n, silu), pw, stats_out=st2)
    assert rel_err(y1.float().cpu(), y2.float().cpu()) < 1e-2
    assert rel_err(st1.cpu(), st2.cpu()) < 1e-2
    # the fold really is the row-block path where it applies
    d = _lib.ConvDesc()
    d.x1, d.C1, d.ld1, d.n_img, d.H, d.W, d.Ho, d.Wo, d.ksize, d.stride = x.data_ptr(), K, K, n, H, H, H, H, 1, 1
    d.aff_scale, d.aff_shift, d.imgs_per_sample = sc.data_ptr(), sh.data_ptr(), 1
    d.w, d.K, d.N, d.y, d.ldy = pw.w.data_ptr(), pw.K, pw.N, y1.data_ptr(), N
    d.row_stats_out = st1.data_ptr()
    assert _lib.load().ls_conv_path(ctypes.byref(d)) == (1 if K in (320, 640) else 2)


@pytest.mark.parametrize("M", [128, 1000, 8192])
def test_feedforward_fused(gpu, M):
    """ls_feedforward (C = 320): y = x + W2 GEGLU(W1 LN(x) + b1) + b2 against the fp32
    reference (diffusers FeedForward / GEGLU after nn.LayerNorm, attention.py:174-199),
    ragged row counts, and against the unfused path (GEGLU row-block GEMM + W2 GEMM)."""
    from latentsync_amd.unet import _Dev, _ff
    from latentsync_amd.packing import pack_ff_w2
    C, I = 320, 1280
    x = bf(rnd(M, C, seed=80) * 2 + 0.5)
    gamma, beta = 1 + 0.2 * rnd(C, seed=81), 0.1 * rnd(C, seed=82)
    w1, b1 = rnd(2 * I, C, seed=83, scale=1 / math.sqrt(C)), rnd(2 * I, seed=84, scale=0.1)
    w2, b2 = rnd(C, I, seed=85, scale=1 / math.sqrt(I)), rnd(C, seed=86, scale=0.1)
    xn = F.layer_norm(x, (C,), gamma, beta, eps=1e-5)
    hg = xn @ w1.T + b1
    ref = x + (hg[:, :I] * F.gelu(hg[:, I:])) @ w2.T + b2
    dv = _Dev({"w2": w2, "b2": b2}, DEV)
    ff1 = dv.packed_ln(w1, b1, (gamma, beta), geglu=True)
    ff2 = dv.packed("w2", "b2")
    ff2p = pack_ff_w2(w2).to(torch.bfloat16).to(DEV)
    xd = x.to(torch.bfloat16).to(DEV)
    st = ops.row_stats(xd)
    assert ops.feedforward_ok(xd, ff1, ff2)
    y = ops.feedforward(xd, st, ff1, ff2, ff2p).float().cpu()
    y2 = _ff(xd, st, ff1, ff2, None).float().cpu()
    assert rel_err(y - x, ref - x) < 2e-2
    assert rel_err(y, y2) < 1e-2


@pytest.mark.parametrize("fm2", [1, 0])
def test_rowblock640_affine_odd_sample_rows(gpu, fm2):
    """K = 640 1x1 conv with the GroupNorm affine folded into the row-block A rows, where a
    sample spans 384 rows (128 x odd): a 256-row block (the two-fragment K = 640 form,
    tuning key 15) would straddle two samples and apply one sample's affine to both, so
    that form must not take RB_AFF -- checked against fp32 per sample and
    against the tiled path with the affine materialised."""
    from latentsync_amd import _lib
    lib = _lib.load()
    n, H, W, C, N = 16, 16, 24, 640, 640   # 384 pixels per sample (imgs_per_sample 1)
    x = bf(rnd(n, H, W, C, seed=120) * 2 + 0.5)
    w = rnd(N, C, seed=121, scale=1 / math.sqrt(C))
    b = rnd(N, seed=122, scale=0.1)
    scale = 1 + 0.3 * rnd(n, C, seed=123)
    shift = 0.5 * rnd(n, C, seed=124)
    pk = packed(w, b, 1)
    xd = x.to(torch.bfloat16).to(DEV)
    aff = (scale.to(DEV), shift.to(DEV), 1, False)
    assert lib.ls_set_tuning(15, fm2) == 0
    try:
        y = ops.conv(xd, pk, aff=aff, aff_materialize=True).float().cpu()
        lib.ls_set_tuning(6, 0)
        try:
            y_tiled = ops.conv(xd, pk, aff=aff, aff_materialize=True).float().cpu()
        finally:
            lib.ls_set_tuning(6, 1)
    finally:
        lib.ls_set_tuning(15, 1)
    ref = bf(x * scale[:, None, None, :] + shift[:, None, None, :]) @ w.T + b
    per_sample = [rel_err(y[i], ref[i]) for i in range(n)]
    print("row-block K=640 affine, per-sample rel_err max", max(per_sample))
    assert max(per_sample) < 1e-2
    assert rel_err(y, y_tiled) < 1e-2


@pytest.mark.parametrize("fmr", [1, 2])
@pytest.mark.parametrize("M", [128 * 3, 65536, 786432])
def test_ff_chain(gpu, M, fmr):
    """ls_ff_chain: h2 = o Wo^T + bo + h1, z = (h2 + FF(LN(h2))) Wp^T + bp + xb in one launch
    (attention.py:174-199 to_out + norm3 + ff, :110-118 proj_out; motion_module.py:126-151,
    262-313) against fp32 with the unfused path's bf16 roundings (h2, LN(h2), GEGLU, y), and
    against the unfused GPU path (row-block to_out with row statistics, ls_feedforward,
    row-block proj_out with GroupNorm column sums): z and its column sums.  M = 786432 is
    the bench's 32x32 level (48 windows).  The fp32 check runs on 4096 rows."""
    from latentsync_amd.unet import _Dev, _ff
    from latentsync_amd.packing import pack_ff_w2
    C, I = 320, 1280
    g = torch.Generator().manual_seed(M)
    r = lambda *s, sc=1.0: torch.randn(*s, generator=g) * sc
    o = bf(r(M, C))
    h1 = bf(r(M, C) * 2 + 0.3)
    xb = bf(r(M, C))
    wo, bo = r(C, C, sc=1 / math.sqrt(C)), r(C, sc=0.1)
    gamma, beta = 1 + 0.2 * r(C), 0.1 * r(C)
    w1, b1 = r(2 * I, C, sc=1 / math.sqrt(C)), r(2 * I, sc=0.1)
    w2, b2 = r(C, I, sc=1 / math.sqrt(I)), r(C, sc=0.1)
    wp, bp = r(C, C, sc=1 / math.sqrt(C)), r(C, sc=0.1)
    dv = _Dev({"wo": wo, "bo": bo, "w2": w2, "b2": b2, "wp": wp, "bp": bp}, DEV)
    pko, pkp, ff2 = dv.packed("wo", "bo"), dv.packed("wp", "bp"), dv.packed("w2", "b2")
    ff1 = dv.packed_ln(w1, b1, (gamma, beta), geglu=True)
    chain = ops.pack_ff_chain(pko, ff1, ff2, pkp)
    od, h1d, xbd = (t.to(torch.bfloat16).to(DEV) for t in (o, h1, xb))
    assert ops.ff_chain_ok(od, chain)
    from latentsync_amd import _lib
    lib = _lib.load()
    if lib.ls_set_tuning(17, fmr) != 0:  # rows per wave: 16 (default) / 32 (diagnostics build)
        pytest.skip("32 rows per wave: diagnostics build only")
    try:
        z = ops.ff_chain(od, h1d, xbd, chain)
    finally:
        lib.ls_set_tuning(17, 1)
    cs = z.gn_cs
    # unfused GPU path
    st = torch.empty((M, 2), dtype=torch.float32, device=DEV)
    h2 = ops.linear(od, pko, res=h1d, stats_out=st)
    y = _ff(h2, st, ff1, ff2, pack_ff_w2(w2).to(torch.bfloat16).to(DEV))
    z2 = ops.conv(y.view(1, 1, M, C), pkp, res=xbd.view(1, 1, M, C), gn_out=True)
    e2 = rel_err(z.float(), z2.view(M, C).float())
    ecs = rel_err(cs.double().sum(0), z2.gn_cs.double().sum(0))
    print(f"ff_chain M={M} fmr={fmr}: vs unfused GPU path rel {e2:.2e}, column sums rel {ecs:.2e}")
    assert e2 < 1e-2 and ecs < 1e-2
    # column sums are those of the stored z (per 128-row slot)
    zz = z.float().view(M // 128, 128, C)
    assert torch.allclose(cs[:, 0], zz.sum(1), rtol=1e-3, atol=1e-2)
    assert torch.allclose(cs[:, 1], (zz * zz).sum(1), rtol=1e-3, atol=1e-1)
    # fp32 reference with the unfused path's bf16 roundings, on the first rows
    n = min(M, 4096)
    h2r = bf(o[:n] @ bf(wo).T + bo + h1[:n])
    t = bf(F.layer_norm(h2r, (C,), gamma, beta, eps=1e-5))
    hg = t @ w1.T + b1
    yr = bf(h2r + bf(hg[:, :I] * F.gelu(hg[:, I:])) @ w2.T + b2)
    zr = yr @ bf(wp).T + bp + xb[:n]
    e = rel_err(z[:n].float().cpu(), zr)
    print(f"ff_chain M={M}: vs fp32 rel {e:.2e}")
    assert e < 1e-2
