"""Thin torch-tensor wrappers over the C-ABI (include/ls_hip.h).

Tensors are device buffers owned by the caller (torch caching allocator); the
wrappers only compute shapes, fill the descriptors and launch on the current
HIP stream, so every call is capturable in a hipGraph (torch.cuda.CUDAGraph).
Activations are NHWC bf16: (images, H, W, C) with frames folded into images.
"""
import ctypes as C
import math

import torch

from . import _lib
from ._lib import check

ACT_NONE, ACT_GEGLU, ACT_GELU, ACT_SILU = 0, 1, 2, 3
_GN_EPILOGUE = _lib.ab_switch("LS_GN_EPILOGUE", "1") != "0"  # A/B switch (diagnostics): 0 = GN stats by read pass
GN_SLOT_ROWS = 128  # LS_GN_SLOT_ROWS


def _p(t):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


class Workspace:
    """Fixed-size per-device scratch (split-K partials, GroupNorm partials).  Never
    re-allocated after creation so captured graphs keep valid pointers."""

    def __init__(self, device, gemm_bytes=256 << 20, gn_bytes=24 << 20):
        self.gemm = torch.empty(gemm_bytes, dtype=torch.uint8, device=device)
        self.gn = torch.zeros(gn_bytes, dtype=torch.uint8, device=device)  # GN arrival counters start at 0


_WS = {}


def workspace(device) -> Workspace:
    key = torch.device(device).index or 0
    if key not in _WS:
        _WS[key] = Workspace(device)
    return _WS[key]


class Packed:
    """A contraction operand ready for ls_conv2d: w bf16 [N][K] (tap-major,
    K padded to 64), bias fp32 [N] or None."""

    def __init__(self, w, bias, cin, ksize, n_out, geglu=False):
        self.w, self.bias, self.cin, self.ksize = w, bias, cin, ksize
        self.N, self.K = w.shape
        self.n_out = n_out
        self.geglu = geglu
        self.colsum = None  # set for LayerNorm-folded weights (unet._Dev.packed_ln)
        self.pe_rows = None  # W pe table for a folded LayerNorm + positional encoding


def _ld(t):
    """Pixel stride of an NHWC view (n, H, W, C): pixel p = (img*H + y)*W + x must
    live at p * ld (channels contiguous)."""
    n, H, W, C_ = t.shape
    st = t.stride()
    ld = st[2] if W > 1 else (st[1] if H > 1 else (st[0] if n > 1 else C_))
    ok = (C_ == 1 or st[3] == 1) and (W == 1 or st[2] == ld) and (H == 1 or st[1] == W * ld) and \
        (n == 1 or st[0] == H * W * ld)
    if not ok:
        raise ValueError(f"NHWC view with non-uniform pixel strides {tuple(st)} for shape {tuple(t.shape)}")
    return ld


def conv_path(x, pw: Packed, **kw):
    """Which kernel family ls_conv2d takes for this call (ls_conv_path: 0 tiled, 1 row-block,
    2 register-staged, 3 halo-tile 3x3) -- host only, nothing is launched."""
    return conv(x, pw, _path_only=True, **kw)


def conv(x, pw: Packed, *, x2=None, aff=None, stride=1, pad=None, upsample=False, out_hw=None, rowvec=None,
         res=None, out_scale=1.0, act=ACT_NONE, out=None, out_f32=False, split_k=0, ln_stats=None,
         stats_out=None, gn_out=False, aff_materialize=False, _path_only=False):
    """Fused conv/linear.  x (n, H, W, C1) [+ x2 (n, H, W, C2)] -> (n, Ho, Wo, n_out).
    aff = (scale[S][C], shift[S][C], imgs_per_sample, silu); rowvec = (t[S][ld], rows_per_vec, ld[, mod]);
    ln_stats = (mean, rstd) rows from row_stats(): LayerNorm folded into pw (pw.colsum);
    stats_out = fp32 (rows, 2) receiving row_stats() of the output (eps 1e-5);
    gn_out = also emit the output's GroupNorm column sums (ls_conv_desc.gn_colsum_out),
    attached to the result as `.gn_cs` for group_norm() (when rows % 128 == 0);
    aff_materialize = when the call would take the register-staged GEMM for the affine
    prologue (ls_conv_path 2), apply it with ls_groupnorm_apply first instead (the
    row-block GEMM folds it into its register-resident A rows)."""
    lib = _lib.load()
    n, H, W, C1 = x.shape
    C2 = x2.shape[3] if x2 is not None else 0
    assert C1 + C2 == pw.cin, (C1, C2, pw.cin)
    ks = pw.ksize
    if pad is None:
        pad = 1 if ks == 3 else 0
    if out_hw is not None:
        Ho, Wo = out_hw
    elif ks == 1:
        Ho, Wo = H, W
    else:
        He, We = (2 * H, 2 * W) if upsample else (H, W)
        Ho, Wo = (He + 2 * pad - 3) // stride + 1, (We + 2 * pad - 3) // stride + 1
    n_out = pw.n_out if act != ACT_GEGLU else pw.N // 2
    if out is None:
        out = torch.empty((n, Ho, Wo, n_out), dtype=torch.float32 if out_f32 else torch.bfloat16, device=x.device)
    ws = workspace(x.device)
    d = _lib.ConvDesc()
    d.x1, d.x2, d.C1, d.C2 = _p(x), _p(x2), C1, C2
    d.ld1, d.ld2 = _ld(x), (_ld(x2) if x2 is not None else 0)
    d.n_img, d.H, d.W, d.Ho, d.Wo = n, H, W, Ho, Wo
    d.ksize, d.stride, d.pad, d.upsample = ks, stride, pad, int(upsample)
    if aff is not None:
        d.aff_scale, d.aff_shift, d.imgs_per_sample, d.silu_in = _p(aff[0]), _p(aff[1]), aff[2], int(aff[3])
    d.w, d.K, d.N = _p(pw.w), pw.K, pw.N
    d.bias = _p(pw.bias)
    if rowvec is not None:
        d.rowvec, d.rows_per_vec, d.rowvec_ld = _p(rowvec[0]), rowvec[1], rowvec[2]
        d.rowvec_mod = rowvec[3] if len(rowvec) > 3 else 0
    if ln_stats is not None:
        assert pw.colsum is not None, "ln_stats needs LayerNorm-folded weights"
        d.ln_rowstats, d.ln_colsum = _p(ln_stats), _p(pw.colsum)
    if res is not None:
        d.res, d.ldr = _p(res), (_ld(res) if res.dim() == 4 else res.stride(-2))
    d.out_scale = out_scale
    d.act = act
    assert tuple(out.shape) == (n, Ho, Wo, n_out), (tuple(out.shape), (n, Ho, Wo, n_out))
    d.y, d.ldy, d.y_f32 = _p(out), _ld(out), int(out.dtype == torch.float32)
    d.split_k = split_k
    if stats_out is not None:
        assert stats_out.dtype == torch.float32 and stats_out.is_contiguous() and stats_out.numel() == 2 * n * Ho * Wo
        assert pw.n_out == pw.N and act != ACT_GEGLU, "row statistics over the real output channels only"
        d.row_stats_out, d.row_stats_eps = _p(stats_out), 1e-5
    if _path_only:
        return lib.ls_conv_path(C.byref(d))
    if aff is not None and aff_materialize and lib.ls_conv_path(C.byref(d)) == 2:
        xa = group_norm_apply(x, aff[0], aff[1], n // aff[2], bool(aff[3]), x2=x2)
        return conv(xa, pw, stride=stride, pad=pad, upsample=upsample, out_hw=out_hw, rowvec=rowvec, res=res,
                    out_scale=out_scale, act=act, out=out, out_f32=out_f32, split_k=split_k, ln_stats=ln_stats,
                    stats_out=stats_out, gn_out=gn_out)
    cs = None
    if gn_out and _GN_EPILOGUE and (n * Ho * Wo) % GN_SLOT_ROWS == 0 and out.dtype == torch.bfloat16 and act != ACT_GEGLU:
        assert pw.n_out == pw.N
        cs = torch.empty((n * Ho * Wo // GN_SLOT_ROWS, 2, n_out), dtype=torch.float32, device=x.device)
        d.gn_colsum_out = _p(cs)
    d.workspace, d.workspace_bytes = _p(ws.gemm), ws.gemm.numel()
    check(lib.ls_conv2d(C.byref(d), _stream()), "ls_conv2d")
    if cs is not None:
        out.gn_cs = cs
    return out


def linear(x2d, pw: Packed, **kw):
    """Token-row linear: x2d (rows, C) -> (rows, n_out).  x2d / res / out may be
    row-strided views (stride(1) == 1)."""
    rows = x2d.shape[0]
    for k in ("res", "out"):
        if kw.get(k) is not None and kw[k].dim() == 2:
            kw[k] = kw[k].unsqueeze(0).unsqueeze(0)
    y = conv(x2d.unsqueeze(0).unsqueeze(0), pw, **kw)
    return y.view(rows, y.shape[-1]) if y.is_contiguous() else y[0, 0]


def gn_colsum(x):
    """Column sums of an existing NHWC bf16 activation (ls_gn_colsum), attached as
    x.gn_cs -- for GroupNorm inputs no GEMM epilogue produced."""
    lib = _lib.load()
    C_ = x.shape[-1]
    rows = x.numel() // C_
    cs = torch.empty((rows // GN_SLOT_ROWS, 2, C_), dtype=torch.float32, device=x.device)
    check(lib.ls_gn_colsum(_p(x), C_, rows, C_, _p(cs), _stream()), "ls_gn_colsum")
    x.gn_cs = cs
    return cs


def _colsums(x, pps):
    cs = getattr(x, "gn_cs", None)
    if cs is None or pps % GN_SLOT_ROWS or not x.is_contiguous():
        return None
    C_ = x.shape[-1]
    return cs if tuple(cs.shape) == (x.numel() // C_ // GN_SLOT_ROWS, 2, C_) else None


def group_norm(x, groups, eps, gamma, beta, n_samples, x2=None):
    """GroupNorm statistics -> (scale, shift) fp32 [n_samples][C].  From the producer's
    column sums (x.gn_cs, conv(..., gn_out=True)) when present, else a read pass."""
    lib = _lib.load()
    C1 = x.shape[-1]
    C2 = x2.shape[-1] if x2 is not None else 0
    pps = x.numel() // C1 // n_samples
    scale = torch.empty((n_samples, C1 + C2), dtype=torch.float32, device=x.device)
    shift = torch.empty_like(scale)
    cs1 = _colsums(x, pps)
    cs2 = _colsums(x2, pps) if x2 is not None else None
    if cs1 is not None and (x2 is None or cs2 is not None):
        check(lib.ls_groupnorm_colsum(_p(cs1), _p(cs2), C1, C2, n_samples, pps, groups, eps, _p(gamma), _p(beta),
                                      _p(scale), _p(shift), _stream()), "ls_groupnorm_colsum")
        return scale, shift
    ws = workspace(x.device)
    check(lib.ls_groupnorm(_p(x), _p(x2), C1, C2, n_samples, pps, groups, eps, _p(gamma), _p(beta), _p(scale),
                           _p(shift), _p(ws.gn), ws.gn.numel(), _stream()), "ls_groupnorm")
    return scale, shift


def group_norm_apply(x, scale, shift, n_samples, silu, x2=None):
    """Materialise act(GN(x | x2)) -> (n, H, W, C1 + C2) bf16."""
    lib = _lib.load()
    C1 = x.shape[-1]
    C2 = x2.shape[-1] if x2 is not None else 0
    n_pix = x.numel() // C1
    y = torch.empty(x.shape[:-1] + (C1 + C2,), dtype=torch.bfloat16, device=x.device)
    check(lib.ls_groupnorm_apply(_p(x), _p(x2), C1, C2, n_pix, n_pix // n_samples, _p(scale), _p(shift), int(silu),
                                 _p(y), _stream()), "ls_groupnorm_apply")
    return y


def affine_act(x, scale, shift, n_samples, silu):
    return group_norm_apply(x, scale, shift, n_samples, silu)


def row_stats(x2d, eps=1e-5):
    """(mean, rstd) fp32 per row of x2d (rows, C) (row-strided views allowed)."""
    lib = _lib.load()
    rows, C_ = x2d.shape
    assert x2d.stride(1) == 1
    st = torch.empty((rows, 2), dtype=torch.float32, device=x2d.device)
    check(lib.ls_row_stats(_p(x2d), x2d.stride(0), rows, C_, eps, _p(st), _stream()), "ls_row_stats")
    return st


def layer_norm(x2d, gamma, beta, eps=1e-5, pe=None, pe_rows_per_frame=1, pe_frames=1):
    """x2d (rows, C), rows may be strided (x2d.stride(1) == 1); y dense (rows, C)."""
    lib = _lib.load()
    rows, C_ = x2d.shape
    assert x2d.stride(1) == 1
    y = torch.empty((rows, C_), dtype=x2d.dtype, device=x2d.device)
    check(lib.ls_layernorm(_p(x2d), x2d.stride(0), rows, C_, eps, _p(gamma), _p(beta), _p(pe), pe_rows_per_frame, pe_frames, _p(y),
                           _stream()), "ls_layernorm")
    return y


def attention(q, k, v, o, *, batch, z2, heads, nq, nk, head_dim, qs, ks, vs, os_, scale=None, fp8=False,
              fp8_workspace=None):
    """qs/ks/vs/os_ = (sb1, sb2, si, sh) element strides; q/k/v/o base tensors
    (may be offset views).  fp8=True: ls_attention_fp8 (P V on the block-scaled e4m3
    MFMA, configs[4]); its V quantisation lands in `fp8_workspace` (uint8, allocated
    here when None -- tests pass their own to read it back)."""
    lib = _lib.load()
    d = _lib.AttnDesc()
    d.q, d.k, d.v, d.o = _p(q), _p(k), _p(v), _p(o)
    for t, st in zip("qkvo", (qs, ks, vs, os_)):
        for name, val in zip(("sb1", "sb2", "si", "sh"), st):
            setattr(d, f"{t}_{name}", int(val))
    d.batch, d.z2, d.heads, d.nq, d.nk, d.head_dim = batch, z2, heads, nq, nk, head_dim
    d.scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    if fp8:
        n = lib.ls_attention_fp8_workspace_bytes(C.byref(d))
        if n == 0:
            raise ValueError(f"ls_attention_fp8: head_dim {head_dim} unsupported (40, 80)")
        if fp8_workspace is None:
            fp8_workspace = torch.empty(n, dtype=torch.uint8, device=q.device)
        check(lib.ls_attention_fp8(C.byref(d), _p(fp8_workspace), fp8_workspace.numel(), _stream()),
              "ls_attention_fp8")
        return o
    check(lib.ls_attention(C.byref(d), _stream()), "ls_attention")
    return o


class TemporalPack:
    """Packed operands of ls_temporal_attention for one VersatileAttention block."""

    def __init__(self, w, gamma, bpe, C, heads, eps=1e-5):
        self.w, self.gamma, self.bpe, self.C, self.heads, self.eps = w, gamma, bpe, C, heads, eps


def pack_temporal(wq, wk, wv, ln_weight, ln_bias, pe, heads, device):
    """ls_temporal_attention operands (include/ls_hip.h) from the reference tensors of one
    VersatileAttention block and its LayerNorm (motion_module.py:203-218, :262-313):
    q|k|v rows per 80-channel group as (q_t, k_t, v_t) 16-row tiles, the q rows scaled
    by log2(e)/sqrt(d) (the kernel's softmax works in log2 units), gamma, and
    beta + pe[f] for f < 16."""
    C = wq.shape[0]
    d = C // heads
    sc = math.log2(math.e) / math.sqrt(d)
    rows = []
    for g in range(C // 80):
        for t in range(5):  # (q_t, k_t, v_t): 16-channel tiles of the group in turn
            cs = slice(80 * g + 16 * t, 80 * g + 16 * t + 16)
            rows += [wq[cs].float() * sc, wk[cs].float(), wv[cs].float()]
    w = torch.cat(rows).to(torch.bfloat16)
    bpe = ln_bias.float().reshape(1, C).repeat(16, 1)
    if pe is not None:
        n = min(16, pe.shape[0])
        bpe[:n] += pe[:n].float().cpu()
    return TemporalPack(w.to(device).contiguous(), ln_weight.float().to(device).contiguous(),
                        bpe.to(device).contiguous(), C, heads)


def temporal_attention_ok(C, heads, F, S):
    """Shapes ls_temporal_attention takes (else the q|k|v GEMM + ls_attention path)."""
    return heads == 8 and 1 <= F <= 16 and ((C == 320 and S % 16 == 0) or (C == 640 and S % 8 == 0))


def temporal_attention(x2d, pk: TemporalPack, n_samples, F, S, out=None):
    """LayerNorm + pe + q|k|v + temporal SDPA of a motion-module attention block in one
    launch (ls_temporal_attention).  x2d (n_samples*F*S, C) rows "(b f) s" -> o, same rows."""
    lib = _lib.load()
    rows, C_ = x2d.shape
    assert C_ == pk.C and rows == n_samples * F * S and x2d.stride(1) == 1
    if out is None:
        out = torch.empty((rows, C_), dtype=torch.bfloat16, device=x2d.device)
    d = _lib.TAttnDesc()
    d.x, d.ldx, d.gamma, d.bpe, d.w = _p(x2d), x2d.stride(0), _p(pk.gamma), _p(pk.bpe), _p(pk.w)
    d.o, d.ldo = _p(out), out.stride(0)
    d.C, d.heads, d.n_samples, d.F, d.S, d.eps = pk.C, pk.heads, n_samples, F, S, pk.eps
    check(lib.ls_temporal_attention(C.byref(d), _stream()), "ls_temporal_attention")
    return out


def feedforward_ok(x2d, w1: "Packed", w2: "Packed"):
    """Shapes ls_feedforward takes (else the GEGLU row-block GEMM + the W2 GEMM)."""
    return (x2d.shape[1] == 320 and w1.N == 2560 and w1.K == 320 and w1.geglu and w2.N == 320 and w2.K == 1280
            and x2d.stride(1) == 1 and x2d.stride(0) % 8 == 0)


def feedforward(x2d, ln_stats, w1: "Packed", w2: "Packed", w2ff, out=None):
    """y = x + W2 GEGLU(W1 LN(x) + b1) + b2 in one launch (ls_feedforward): x2d (M, 320)
    rows, ln_stats (M, 2) their (mean, rstd); w1 the LN-folded GEGLU operand, w2 the W2
    operand (bias), w2ff = packing.pack_ff_w2(W2) bf16."""
    lib = _lib.load()
    M, C_ = x2d.shape
    if out is None:
        out = torch.empty((M, C_), dtype=torch.bfloat16, device=x2d.device)
    d = _lib.FFDesc()
    d.x, d.ln_rowstats, d.w1, d.b1 = _p(x2d), _p(ln_stats), _p(w1.w), _p(w1.bias)
    d.w2, d.b2, d.y = _p(w2ff), _p(w2.bias), _p(out)
    d.M, d.ldx, d.ldy, d.C, d.inner = M, x2d.stride(0), out.stride(0), C_, w1.N // 2
    check(lib.ls_feedforward(C.byref(d), _stream()), "ls_feedforward")
    return out


class FFChainPack:
    """ls_ff_chain operands of one block tail (packing.pack_ff_chain): to_out, the
    LN-folded GEGLU W1 (k permuted), W2 (pack_ff_w2), proj_out (k permuted)."""

    def __init__(self, wo, bo, w1, b1, w2, b2, wp, bp, C, inner, eps):
        self.wo, self.bo, self.w1, self.b1, self.w2, self.b2, self.wp, self.bp = wo, bo, w1, b1, w2, b2, wp, bp
        self.C, self.inner, self.eps = C, inner, eps


def pack_ff_chain(wo: "Packed", ff1: "Packed", ff2: "Packed", po: "Packed", eps=1e-5):
    """FFChainPack from the packed operands of the unfused path: to_out (C, C) + bias, the
    LN-folded GEGLU W1 (interleaved, gamma folded) + bias, W2 + bias, proj_out + bias."""
    from .packing import pack_ff_w2, permute_k_acc
    Cc = wo.N
    bf = lambda t: t.to(torch.bfloat16).contiguous()
    w1 = permute_k_acc(ff1.w.float())
    return FFChainPack(bf(pack_ff_w2(wo.w.float()[:, :Cc], permute=False)), wo.bias.float().contiguous(), bf(w1),
                       ff1.bias.float().contiguous(), bf(pack_ff_w2(ff2.w.float()[:, :ff2.K])),
                       ff2.bias.float().contiguous(), bf(pack_ff_w2(po.w.float()[:, :Cc])),
                       po.bias.float().contiguous(), Cc, ff1.N // 2, eps)


def ff_chain_ok(o2d, pk: "FFChainPack"):
    return (pk is not None and o2d.shape[1] == 320 and pk.inner == 1280 and o2d.shape[0] % 128 == 0
            and o2d.stride(1) == 1 and o2d.stride(0) % 8 == 0)


def ff_chain(o2d, h1, xb, pk: "FFChainPack", shape=None, gn_out=True):
    """z = proj_out(FF(LN(h2)) + h2) + xb with h2 = to_out(o) + h1, one launch (ls_ff_chain);
    o2d / h1 / xb (M, C) rows; z is allocated with `shape` (default (M, C)) and carries
    .gn_cs (its GroupNorm column sums) for group_norm()."""
    lib = _lib.load()
    M, C_ = o2d.shape
    res = torch.empty(shape or (M, C_), dtype=torch.bfloat16, device=o2d.device)
    out = res.view(M, C_)
    cs = torch.empty((M // GN_SLOT_ROWS, 2, C_), dtype=torch.float32, device=o2d.device) if gn_out else None
    d = _lib.FFChainDesc()
    d.o, d.wo, d.bo, d.h1 = _p(o2d), _p(pk.wo), _p(pk.bo), _p(h1)
    d.w1, d.b1, d.w2, d.b2, d.wp, d.bp = _p(pk.w1), _p(pk.b1), _p(pk.w2), _p(pk.b2), _p(pk.wp), _p(pk.bp)
    d.xb, d.z, d.cs_out = _p(xb), _p(out), _p(cs)
    d.M, d.ldo, d.ldh, d.ldxb, d.ldz = M, o2d.stride(0), h1.stride(0), xb.stride(0), out.stride(0)
    d.C, d.inner, d.eps = C_, pk.inner, float(pk.eps)
    check(lib.ls_ff_chain(C.byref(d), _stream()), "ls_ff_chain")
    if cs is not None:
        res.gn_cs = cs
    return res


class XAttnPack:
    """ls_cross_attention_block operands of one BasicTransformerBlock's attn2 + norm2
    (packing.pack_xattn_q / pack_xattn_wo)."""

    def __init__(self, wq, bq, wo, bo, C, heads):
        self.wq, self.bq, self.wo, self.bo, self.C, self.heads = wq, bq, wo, bo, C, heads


def pack_cross_attention(wq, ln_weight, ln_bias, wo, bo, heads, device):
    """XAttnPack from the reference tensors: to_q.weight (C, C), norm2 gamma / beta,
    to_out.0.weight (C, C) / bias -- LayerNorm folded (W gamma, W beta) in fp32 before the
    single bf16 rounding."""
    from .packing import pack_xattn_q, pack_xattn_wo
    w = wq.float().cpu()
    gamma, beta = ln_weight.float().cpu(), ln_bias.float().cpu()
    pq, pb = pack_xattn_q(w * gamma[None, :], w @ beta, heads)
    po = pack_xattn_wo(wo.float().cpu(), heads)
    bf = lambda t: t.to(torch.bfloat16).to(device).contiguous()
    return XAttnPack(bf(pq), pb.to(device).contiguous(), bf(po), bo.float().to(device).contiguous(), w.shape[0], heads)


def cross_attention_ok(x2d, pk, L, hw):
    """Shapes ls_cross_attention_block takes (else q GEMM + ls_attention + out GEMM)."""
    return (pk is not None and x2d.shape[1] == 320 and pk.heads == 8 and 1 <= L <= 64 and hw % 128 == 0
            and x2d.shape[0] % hw == 0 and x2d.stride(1) == 1 and x2d.stride(0) % 8 == 0)


def cross_attention_block(x2d, ln_stats, pk: XAttnPack, kv, L, hw, stats_out, out=None, eps=1e-5):
    """y = x + to_out(attn(to_q(LN(x)), k, v)) for the audio cross attention in one launch
    (ls_cross_attention_block); stats_out (M, 2) receives y's LayerNorm row statistics."""
    lib = _lib.load()
    M, C_ = x2d.shape
    if out is None:
        out = torch.empty((M, C_), dtype=torch.bfloat16, device=x2d.device)
    assert stats_out.dtype == torch.float32 and stats_out.is_contiguous() and stats_out.numel() == 2 * M
    assert kv.stride(1) == 1 and kv.shape[0] == (M // hw) * L and kv.shape[1] >= 2 * C_
    d = _lib.XAttnDesc()
    d.x, d.ln_rowstats, d.wq, d.bq, d.kv, d.wo, d.bo = _p(x2d), _p(ln_stats), _p(pk.wq), _p(pk.bq), _p(kv), \
        _p(pk.wo), _p(pk.bo)
    d.y, d.stats_out = _p(out), _p(stats_out)
    d.M, d.ldx, d.ldy, d.ldkv, d.C, d.heads, d.L, d.hw, d.eps = M, x2d.stride(0), out.stride(0), kv.stride(0), C_, \
        pk.heads, L, hw, eps
    check(lib.ls_cross_attention_block(C.byref(d), _stream()), "ls_cross_attention_block")
    return out


def attention_fp8_workspace_bytes(*, batch, heads, nk, head_dim):
    lib = _lib.load()
    d = _lib.AttnDesc()
    d.batch, d.z2, d.heads, d.nq, d.nk, d.head_dim = batch, 1, heads, 1, nk, head_dim
    return lib.ls_attention_fp8_workspace_bytes(C.byref(d))


def small_linear(x, w, bias, silu_in=False, out=None):
    lib = _lib.load()
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=x.device)
    check(lib.ls_small_linear(_p(x), M, K, _p(w), _p(bias), N, int(silu_in), _p(out), _stream()), "ls_small_linear")
    return out


def timestep_embed(timesteps_i32, step_i32, B, dim, flip=True, shift=0.0, out=None):
    lib = _lib.load()
    if out is None:
        out = torch.empty((B, dim), dtype=torch.float32, device=timesteps_i32.device)
    check(lib.ls_timestep_embed(_p(timesteps_i32), _p(step_i32), B, dim, int(flip), float(shift), _p(out), _stream()),
          "ls_timestep_embed")
    return out


def timestep_embed_f32(t_f32, dim, flip=True, shift=0.0, out=None):
    """One embedding row per fp32 timestep (forward()'s float / per-sample timesteps)."""
    lib = _lib.load()
    B = t_f32.numel()
    if out is None:
        out = torch.empty((B, dim), dtype=torch.float32, device=t_f32.device)
    check(lib.ls_timestep_embed_f32(_p(t_f32), B, dim, int(flip), float(shift), _p(out), _stream()),
          "ls_timestep_embed_f32")
    return out


def ddim_cfg_step(eps, Bu, guidance, lat, coef, step, unet_in):
    lib = _lib.load()
    P = lat.shape[0]
    check(lib.ls_ddim_cfg_step(_p(eps), eps.shape[-1], Bu, P, float(guidance), _p(lat), _p(coef), _p(step),
                               _p(unet_in), unet_in.shape[-1], _stream()), "ls_ddim_cfg_step")


def prep_pixels(faces_u8, mask, ld=8, pix=None, masked=None):
    lib = _lib.load()
    F_, _, R, _ = faces_u8.shape
    if pix is None:
        pix = torch.empty((F_, R, R, ld), dtype=torch.bfloat16, device=faces_u8.device)
    if masked is None:
        masked = torch.empty_like(pix)
    check(lib.ls_prep_pixels(_p(faces_u8), F_, R, _p(mask), _p(pix), _p(masked), ld, _stream()), "ls_prep_pixels")
    return pix, masked


def vae_sample(moments, eps, scaling, shift, dst, c_off):
    lib = _lib.load()
    P = eps.shape[0]
    check(lib.ls_vae_sample(_p(moments), moments.shape[-1], _p(eps), P, float(scaling), float(shift), _p(dst),
                            dst.shape[-1], c_off, _stream()), "ls_vae_sample")


def pack_unet_input(lat, cond, mask, F_, R, h, Bu, unet_in):
    lib = _lib.load()
    check(lib.ls_pack_unet_input(_p(lat), _p(cond), _p(mask), F_, R, h, Bu, _p(unet_in), unet_in.shape[-1],
                                 _stream()), "ls_pack_unet_input")


def scale_latents(lat, inv_scaling, shift, z):
    lib = _lib.load()
    check(lib.ls_scale_latents(_p(lat), lat.shape[0], float(inv_scaling), float(shift), _p(z), z.shape[-1],
                               _stream()), "ls_scale_latents")


def paste_back(dec, pix, mask, out_nchw=None, out_u8=None):
    lib = _lib.load()
    F_, R = dec.shape[0], dec.shape[1]
    check(lib.ls_paste_back(_p(dec), dec.shape[-1], _p(pix), pix.shape[-1], _p(mask), F_, R, _p(out_nchw),
                            _p(out_u8), _stream()), "ls_paste_back")


def add_rows(x2d, table, out=None):
    lib = _lib.load()
    rows, C_ = x2d.shape
    if out is None:
        out = torch.empty_like(x2d)
    check(lib.ls_add_rows(_p(x2d), rows, C_, x2d.stride(0), _p(table), table.shape[0], _p(out), out.stride(0),
                          _stream()), "ls_add_rows")
    return out
