"""CPU restatement of the fp8 attention path (ls_attention_fp8) -- TEST INFRASTRUCTURE.

Only tests/ (and bench.py's cpu_baseline leg, which does not use this file) may
import it; the product path runs on libls_hip.so alone.

The reference has no fp8 path: LatentSync runs F.scaled_dot_product_attention in
fp16/fp32 (latentsync/models/attention.py:271).  BASELINE.json configs[4] asks for
"fp8 MFMA attention", so this file restates the quantisation the kernel applies and
the attention it then computes; the anchor for the fp8 result against the reference
is fp32 SDPA with the tolerance stated in tests/test_gpu_fp8.py.

  * V quantisation (vt8_quant_kernel, latentsync_amd/csrc/ls_attn.hip): per
    (batch, head) the keys are cut into 128-key tiles; inside a tile, head dim d and
    lane group lg own the 32 keys 16 (j >> 2) + 4 lg + (j & 3), j = 0..31 (the keys
    a 16x16x128 MFMA lane group holds).  One e8m0 scale per (d, tile), stored once per
    lane group: e = floor(log2(amax)) - 7 over the tile's 128 keys (amax = 0: e = -127),
    clamped to e + 127 in [0, 254]; values are stored as e4m3fn(v * 2^-e) (OCP, round
    to nearest even).
  * Attention: Q pre-scaled by scale * log2(e) and rounded to bf16 (as the kernel
    does), scores in fp32, p = e4m3(2^(s - m)) with m = ceil(row max) - 7 (the row's
    largest p in (2^6, 2^7], so e4m3's normal range covers 13 binades below it),
    O = p V_q / sum p with V_q the dequantised V.  The kernel's m is such an integer
    too, taken at the last tile that moved it (by more than 8), so its p are these
    times 2^k, k in {0, 1}, which e4m3 rounds identically outside the subnormal range:
    the emulation matches it to fp32-accumulation noise.
"""
import torch

KT = 128  # keys per tile


def key_perm():
    """pos = 32 lg + j -> key offset inside the tile."""
    pos = torch.arange(KT)
    lg, j = pos // 32, pos % 32
    return 16 * (j // 4) + 4 * lg + (j % 4)


def quant_vt(v):
    """v: fp32 [nk, D] (bf16 values) of one (batch, head).  Returns
    (codes uint8 [ntile, D, 128] in position order, e8 uint8 [ntile, D, 4])."""
    nk, D = v.shape
    nt = (nk + KT - 1) // KT
    vp = torch.zeros(nt * KT, D, dtype=torch.float32)
    vp[:nk] = v.float()
    vt = vp.view(nt, KT, D).permute(0, 2, 1)[:, :, key_perm()]  # [nt, D, 128] position order
    blk = vt.reshape(nt, D, 4, 32)
    amax = blk.abs().amax((-2, -1), keepdim=True).squeeze(-1).expand(nt, D, 4)
    _, ex = torch.frexp(amax)                      # amax = m 2^ex, m in [0.5, 1)
    e = torch.where(amax > 0, ex - 1 - 7, torch.full_like(ex, -127))
    e8 = (e + 127).clamp(0, 254)
    e = e8 - 127
    scaled = blk * torch.pow(2.0, -e.double()).float().unsqueeze(-1)
    codes = scaled.to(torch.float8_e4m3fn).view(torch.uint8).reshape(nt, D, KT)
    return codes, e8.to(torch.uint8)


def dequant_vt(codes, e8, nk):
    """Inverse of quant_vt: fp32 V_q [nk, D]."""
    nt, D, _ = codes.shape
    vals = codes.view(torch.float8_e4m3fn).float().view(nt, D, 4, 32)
    vals = vals * torch.pow(2.0, e8.double() - 127).float().unsqueeze(-1)
    vt = torch.empty(nt, D, KT)
    vt[:, :, key_perm()] = vals.reshape(nt, D, KT)
    return vt.permute(0, 2, 1).reshape(nt * KT, D)[:nk]


def attention_fp8(q, k, v, scale):
    """q [nq, D], k/v [nk, D] fp32 (bf16 values) of one (batch, head) -> fp32 [nq, D]."""
    c2 = scale * 1.4426950408889634
    qs = (q.float() * c2).to(torch.bfloat16).float()
    s = qs @ k.float().t()
    p = torch.exp2(s - (torch.ceil(s.amax(-1, keepdim=True)) - 7)).to(torch.float8_e4m3fn).float()
    codes, e8 = quant_vt(v)
    vq = dequant_vt(codes, e8, v.shape[0])
    return (p @ vq) / p.sum(-1, keepdim=True)


def decode_workspace(ws, pairs, nk, D):
    """The GPU workspace of ls_attention_fp8 -> (codes [pairs, ntile, ND*16, 128] in
    position order, e8 [pairs, ntile, ND*16, 4]); layout of ls_attn.hip Fp8Tile."""
    ND = (D + 16) // 16
    R = ND * 16
    nsc = (ND + 3) // 4
    vbytes = R * 128
    tb = vbytes + nsc * 256
    nt = (nk + KT - 1) // KT
    t = ws[: pairs * nt * tb].view(pairs, nt, tb)
    raw = t[:, :, :vbytes].reshape(pairs, nt, R, 8, 16)
    d = torch.arange(R)
    c = torch.arange(8)
    phys = c.view(1, 8) ^ ((d.view(R, 1) >> 1) & 7)                         # logical chunk -> stored chunk
    codes = torch.gather(raw, 3, phys.view(1, 1, R, 8, 1).expand(pairs, nt, R, 8, 16)).reshape(pairs, nt, R, 128)
    sc = t[:, :, vbytes:].reshape(pairs, nt, nsc, 64, 4)                     # [blk][lane][byte]
    nd, lq = d // 16, d % 16
    e8 = torch.stack([sc[:, :, nd // 4, lg * 16 + lq, nd % 4] for lg in range(4)], -1)  # [pairs, nt, R, 4]
    return codes, e8
