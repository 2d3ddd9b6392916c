"""Temporal (short-sequence) attention at the bench shapes: the motion module's
'(b f) s c' rows (frame-major, 16 rows per pixel sequence S*3C apart) against the
same data pixel-major ('(b s) f c', a sequence's rows contiguous), input and output
layouts varied independently, plus a device copy of the same bytes as the rate
reference.  usage: python scripts/seq_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from latentsync_amd import ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import timed  # noqa: E402

B, F, H = 16, 16, 8  # configs[1]: 16 windows x 16 frames, latent 32^2
for C, S in ((320, 1024), (640, 256), (1280, 64)):
    d = C // H
    qkv = torch.randn(B * F * S, 3 * C, device="cuda").to(torch.bfloat16)
    o = torch.empty(B * F * S, C, device="cuda", dtype=torch.bfloat16)
    by = 4.0 * B * F * S * C * 2
    fm_in = (F * S * 3 * C, 3 * C, S * 3 * C, d)   # rows (b f s)
    pm_in = (F * S * 3 * C, F * 3 * C, 3 * C, d)   # rows (b s f)
    fm_out = (F * S * C, C, S * C, d)
    pm_out = (F * S * C, F * C, C, d)
    for name, si, so in (("frame-major in/out", fm_in, fm_out), ("pixel-major in/out", pm_in, pm_out),
                         ("frame-major in, pixel-major out", fm_in, pm_out),
                         ("pixel-major in, frame-major out", pm_in, fm_out)):
        t = timed(lambda: ops.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=B * S, z2=S, heads=H, nq=F, nk=F,
                                        head_dim=d, qs=si, ks=si, vs=si, os_=so))
        print(f"C={C:5d} S={S:5d} {name:34s} {t * 1e3:8.1f} us  {by / t / 1e6:7.1f} GB/s", flush=True)
    dst = torch.empty_like(qkv)
    t = timed(lambda: dst.copy_(qkv))
    print(f"C={C:5d} S={S:5d} {'device copy of q|k|v':34s} {t * 1e3:8.1f} us  {2.0 * qkv.numel() * 2 / t / 1e6:7.1f} GB/s",
          flush=True)

# the same call after a MALL flush (1 GiB memset) and after a large GEMM (clock /
# power state of the bench's steps): per-launch HIP events, median of 10
if __name__ == "__main__":
    flush = torch.empty(1 << 29, dtype=torch.int16, device="cuda")
    a = torch.randn(8192, 8192, device="cuda").to(torch.bfloat16)
    for C, S in ((320, 1024), (640, 256)):
        d = C // H
        qkv = torch.randn(B * F * S, 3 * C, device="cuda").to(torch.bfloat16)
        o = torch.empty(B * F * S, C, device="cuda", dtype=torch.bfloat16)
        by = 4.0 * B * F * S * C * 2
        st, so = (F * S * 3 * C, 3 * C, S * 3 * C, d), (F * S * C, C, S * C, d)
        for pre in ("none", "flush", "gemm", "flush+gemm"):
            ts = []
            for _ in range(12):
                if "flush" in pre:
                    flush.fill_(1)
                if "gemm" in pre:
                    torch.mm(a, a)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=B * S, z2=S, heads=H, nq=F, nk=F,
                              head_dim=d, qs=st, ks=st, vs=st, os_=so)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e-3)
            t = sorted(ts[2:])[len(ts[2:]) // 2]
            print(f"C={C:5d} S={S:5d} after {pre:12s} {t * 1e6:8.1f} us  {by / t / 1e9:7.1f} GB/s", flush=True)
