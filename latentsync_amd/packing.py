"""One-time weight packing from reference-named fp32 state dicts to the layouts
the kernels consume (done at load / .to(device), never per step).

  conv / linear  W (O, I[, k, k]) -> bf16 [O][K], K = k*k*I8 rounded up to 64,
                 tap-major (kh, kw, ci), I8 = I rounded up to 8 (zero channels);
                 3x3 with I % 64 == 0: channel-chunk-major (ci / 64, kh, kw, ci % 64)
  GEGLU W1       rows [h(4C); g(4C)] interleaved in 16-row blocks so packed
                 column 32b+i = h_{16b+i}, 32b+16+i = g_{16b+i} (epilogue pairs)
  fused q|k|v    rows concatenated (self-attention shares one LN output)
"""
import torch


def _r8(n):
    return (n + 7) // 8 * 8


def _r64(n):
    return (n + 63) // 64 * 64


def pack_weight(w: torch.Tensor, cin_pad: int = None, n_pad: int = None) -> torch.Tensor:
    """w (O, I) or (O, I, k, k) fp32 -> fp32 (O', K) tap-major, zero padded."""
    w = w.float()
    if w.dim() == 2:
        w = w[:, :, None, None]
    if w.dim() == 3:  # conv1d (O, I, k) -> 3x3 with the kernel on the middle row
        O, I, k = w.shape
        assert k == 3
        w2 = torch.zeros(O, I, 3, 3, dtype=w.dtype)
        w2[:, :, 1, :] = w
        w = w2
    O, I, kh, kw = w.shape
    ip = cin_pad or _r8(I)
    if ip != I:
        w = torch.cat([w, torch.zeros(O, ip - I, kh, kw, dtype=w.dtype)], 1)
    w = w.permute(0, 2, 3, 1)  # (O, kh, kw, ip)
    if kh == 3 and ip % 64 == 0:
        # channel-chunk-major: k = (ci / 64) * 576 + tap * 64 + ci % 64 (the 9 taps of a
        # 64-channel chunk are consecutive K-tiles; ls_conv2d's gather follows, ls_hip.h)
        w = w.reshape(O, 9, ip // 64, 64).permute(0, 2, 1, 3).reshape(O, 9 * ip)
    else:
        w = w.reshape(O, kh * kw * ip)
    K = _r64(w.shape[1])
    if K != w.shape[1]:
        w = torch.cat([w, torch.zeros(O, K - w.shape[1], dtype=w.dtype)], 1)
    if n_pad and n_pad > O:
        w = torch.cat([w, torch.zeros(n_pad - O, K, dtype=w.dtype)], 0)
    return w


def pad_bias(b, n_pad=None):
    if b is None:
        return None
    b = b.float()
    if n_pad and n_pad > b.shape[0]:
        b = torch.cat([b, torch.zeros(n_pad - b.shape[0])])
    return b


def geglu_interleave(w1: torch.Tensor, b1: torch.Tensor):
    """w1 (8C, C) = [h; g] -> rows interleaved in 16-blocks; b1 likewise."""
    n2 = w1.shape[0] // 2
    assert n2 % 16 == 0
    h, g = w1[:n2], w1[n2:]
    w = torch.stack([h.reshape(n2 // 16, 16, -1), g.reshape(n2 // 16, 16, -1)], 1).reshape(2 * n2, -1)
    bh, bg = b1[:n2], b1[n2:]
    b = torch.stack([bh.reshape(-1, 16), bg.reshape(-1, 16)], 1).reshape(-1)
    return w, b


# k-slot (lane group lg, element i) of a 32-wide k-step -> the column a lane holds there after
# a 16x16 MFMA accumulator tile pair (columns 4 lg .. + 3 of tile 0, then of tile 1)
ACC_K_PERM = [(4 * lg + i) if i < 4 else (16 + 4 * lg + i - 4) for lg in range(4) for i in range(8)]


def pack_ff_w2(w2: torch.Tensor, permute: bool = True) -> torch.Tensor:
    """FeedForward W2 (C, I) -> [I/32][C][32] for ls_feedforward (include/ls_hip.h): per
    32-column chunk, k-slot (lg, i) of a row holds column i < 4 ? 4 lg + i : 16 + 4 lg + i - 4
    (the GEGLU values a lane holds after GEMM1), and the row's four 16-B pieces are stored
    at physical piece lg ^ (((row >> 3) & 1) << 1) (conflict-free ds_read_b128).
    permute=False keeps the natural column order (ls_ff_chain's wo: its operand rows come
    from memory)."""
    C, I = w2.shape
    assert I % 32 == 0
    perm = torch.tensor(ACC_K_PERM if permute else list(range(32)))
    w = w2.float().reshape(C, I // 32, 32)[:, :, perm]          # (C, chunk, 32 logical slots)
    w = w.reshape(C, I // 32, 4, 8)                              # (..., logical piece, 8)
    rows = torch.arange(C)
    phys = torch.arange(4)[None, :] ^ (((rows[:, None] >> 3) & 1) << 1)  # logical -> physical piece
    out = torch.empty_like(w)
    out[rows[:, None], :, phys, :] = w.permute(0, 2, 1, 3)       # (C, piece, chunk, 8) scattered
    return out.permute(1, 0, 2, 3).reshape(I // 32, C, 32).contiguous()


def permute_k_acc(w: torch.Tensor) -> torch.Tensor:
    """Columns of a [N][K] operand (K % 32 == 0) permuted within each 32-wide k-step by
    ACC_K_PERM: for a B operand built from MFMA accumulators in registers (ls_ff_chain's W1)."""
    N, K = w.shape
    assert K % 32 == 0
    return w.reshape(N, K // 32, 32)[:, :, torch.tensor(ACC_K_PERM)].reshape(N, K).contiguous()


def _xattn_slot_dims():
    """Head-local (head offset, dim) of every k-slot of the fused cross-attention's
    out-projection (ls_cross_attention_block): k-step 3j + u, lane group lg, element e.
    u = 0, 1: head 2j + u, dims 4 lg + e (e < 4) / 16 + 4 lg + e - 4; u = 2: dims 32 + 4 lg
    + (e & 3) of head 2j (e < 4) / 2j + 1 (e >= 4), lane groups 2, 3 padding (None)."""
    out = []
    for ks in range(12):
        j, u = divmod(ks, 3)
        for lg in range(4):
            for e in range(8):
                if u < 2:
                    out.append((2 * j + u, 4 * lg + e if e < 4 else 16 + 4 * lg + e - 4))
                elif lg < 2:
                    out.append((2 * j + (e >= 4), 32 + 4 * lg + (e & 3)))
                else:
                    out.append(None)
    return out


def pack_xattn_q(wq: torch.Tensor, bq: torch.Tensor, heads: int = 8):
    """to_q with norm2's gamma / beta folded (the LN-folded operand: W (C, C), bias (C))
    -> ls_cross_attention_block's wq [heads][C/64 k-images][48 rows][8 pieces][8] bf16 and
    bq [heads][48] fp32: each head's 40 rows padded to 48 (zero), scaled by log2(e)/sqrt(d)
    (the kernel's softmax works in log2 units), 16-B pieces of a 64-wide k-image stored at
    physical piece lc ^ ((row >> 1) & 7) (the row-block GEMM's swizzle)."""
    import math
    C = wq.shape[0]
    d = C // heads
    sc = math.log2(math.e) / math.sqrt(d)
    w = torch.zeros(heads, 48, C)
    w[:, :d] = wq.float().reshape(heads, d, C) * sc
    b = torch.zeros(heads, 48)
    b[:, :d] = bq.float().reshape(heads, d) * sc
    w = w.reshape(heads, 48, C // 64, 8, 8).permute(0, 2, 1, 3, 4)  # (head, img, row, logical piece, 8)
    rows = torch.arange(48)
    phys = torch.arange(8)[None, :] ^ ((rows[:, None] >> 1) & 7)    # (row, logical) -> physical
    out = torch.empty_like(w)
    out[:, :, rows[:, None], phys, :] = w
    return out.contiguous(), b.contiguous()


def pack_xattn_wo(wo: torch.Tensor, heads: int = 8):
    """to_out (C, C) -> ls_cross_attention_block's wo [C/32 chunks][2 tiles][12 k-steps][16
    rows][4 pieces][8] bf16: column slots in the kernel's o register order
    (_xattn_slot_dims), padding slots zero, the 16-B pieces of a row at physical piece
    lg ^ (((row >> 3) & 1) << 1) (conflict-free ds_read_b128, as pack_ff_w2)."""
    C = wo.shape[0]
    d = C // heads
    idx = torch.tensor([40 * 0 + 0 if s is None else s[0] * d + s[1] for s in _xattn_slot_dims()])
    valid = torch.tensor([s is not None for s in _xattn_slot_dims()])
    w = wo.float()[:, idx] * valid[None, :].float()                  # (C out, 384 slots)
    w = w.reshape(C // 32, 2, 16, 12, 4, 8).permute(0, 1, 3, 2, 4, 5)  # (chunk, tile, ks, row, lg, 8)
    rows = torch.arange(16)
    phys = torch.arange(4)[None, :] ^ (((rows[:, None] >> 3) & 1) << 1)
    out = torch.empty_like(w)
    out[:, :, :, rows[:, None], phys, :] = w
    return out.contiguous()
