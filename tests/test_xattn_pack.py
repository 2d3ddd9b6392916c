"""Host packing of the fused audio cross-attention (ls_cross_attention_block,
packing.pack_xattn_q / pack_xattn_wo), checked on the CPU against the index maps the
kernel reads them with (latentsync_amd/csrc/ls_xattn.hip), and the out-projection's
k-slot scheme end to end: o values placed in the registers the way the kernel places
them, contracted with the packed Wo the way the MFMAs do, equal Wo @ o exactly."""
import math

import torch

from latentsync_amd.packing import _xattn_slot_dims, pack_xattn_q, pack_xattn_wo

C, H, D = 320, 8, 40


def _swz64(row, c):
    return row * 8 + (c ^ ((row >> 1) & 7))


def test_pack_xattn_q_index_map():
    g = torch.Generator().manual_seed(0)
    w, b = torch.randn(C, C, generator=g), torch.randn(C, generator=g)
    pq, pb = pack_xattn_q(w, b, H)
    sc = math.log2(math.e) / math.sqrt(D)
    flat = pq.reshape(H, -1, 8)  # uint4 pieces of 8 values
    for h in (0, 3, 7):
        for t in range(3):
            for s in range(10):
                for l16 in (0, 5, 15):
                    for lg in range(4):
                        got = flat[h, (s >> 1) * 384 + _swz64(t * 16 + l16, (s & 1) * 4 + lg)]
                        r = 16 * t + l16
                        want = w[40 * h + r, 32 * s + 8 * lg:32 * s + 8 * lg + 8] * sc if r < D else torch.zeros(8)
                        assert torch.allclose(got, want, atol=1e-6), (h, t, s, l16, lg)
    assert torch.allclose(pb[:, :D], b.reshape(H, D) * sc) and pb[:, D:].abs().max() == 0


def test_pack_xattn_wo_slot_scheme_end_to_end():
    """The kernel's o registers: per head h, tiles nd of 16 dims, lane group lg holds dims
    16 nd + 4 lg + r; ofr[3(h>>1) + (h&1)] = {nd0 r, nd1 r}, ofr[3(h>>1) + 2][(h&1)*4 + r] = nd2 r
    (lane groups 2, 3 carry the padding dims 40..47, set to garbage here)."""
    g = torch.Generator().manual_seed(1)
    wo = torch.randn(C, C, generator=g)
    o = torch.randn(H, 48, generator=g)  # one row's o, 48 dims per head (40..47 garbage)
    pw = pack_xattn_wo(wo, H).reshape(C // 32, 2, 12, 16, 4, 8)
    ofr = torch.zeros(12, 4, 8)  # [k-step][lane group][element]
    for h in range(H):
        ja, jb, eb = 3 * (h >> 1) + (h & 1), 3 * (h >> 1) + 2, (h & 1) * 4
        for lg in range(4):
            for r in range(4):
                ofr[ja, lg, r] = o[h, 4 * lg + r]
                ofr[ja, lg, 4 + r] = o[h, 16 + 4 * lg + r]
                ofr[jb, lg, eb + r] = o[h, 32 + 4 * lg + r]
    y = torch.zeros(C)
    for c in range(C // 32):
        for t in range(2):
            for l16 in range(16):
                p2 = [lg ^ (((l16 >> 3) & 1) << 1) for lg in range(4)]
                acc = 0.0
                for ks in range(12):
                    for lg in range(4):
                        acc += float((pw[c, t, ks, l16, p2[lg]] * ofr[ks, lg]).sum())
                y[32 * c + 16 * t + l16] = acc
    want = wo @ o[:, :D].reshape(-1)
    assert torch.allclose(y, want, rtol=1e-4, atol=1e-3), (y - want).abs().max()
    # every real dim appears in exactly one slot, the padding slots are the 16 per pair
    dims = [s for s in _xattn_slot_dims() if s is not None]
    assert len(dims) == C and len(set(dims)) == C
