"""Achievable HBM rate on this box for the short-K projections' traffic pattern, without
the GEMM: y = a + r over bf16 tensors of the out0 / out1 / out2 shapes (read two, write
one -- the bytes a K = C residual projection must move), plus a plain copy and a read-only
reduction.  torch's elementwise kernels, hipGraph-replayed, median of 20.
usage: python scripts/hbm_probe.py"""
import torch

dev = torch.device("cuda", 0)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2] * 1e3  # us


for name, M, N in [("out0", 786432, 320), ("out1", 196608, 640), ("out2", 49152, 1280), ("1 GiB", 1 << 20, 512)]:
    a = torch.randn(M, N, device=dev).to(torch.bfloat16)
    r = torch.randn(M, N, device=dev).to(torch.bfloat16)
    y = torch.empty_like(a)
    s = torch.empty(N, device=dev, dtype=torch.float32)
    nb = M * N * 2
    t_add = timed(lambda: torch.add(a, r, out=y))
    t_cp = timed(lambda: y.copy_(a))
    t_sum = timed(lambda: torch.sum(a, dim=0, dtype=torch.float32, out=s))
    print(f"{name:6s} M={M} N={N}: a+r->y {t_add:8.1f} us {3 * nb / t_add / 1e6:6.2f} TB/s | copy {t_cp:8.1f} us "
          f"{2 * nb / t_cp / 1e6:6.2f} TB/s | column sum {t_sum:8.1f} us {nb / t_sum / 1e6:6.2f} TB/s", flush=True)
    del a, r, y
