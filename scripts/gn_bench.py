"""GroupNorm stats / apply micro-benchmark on the UNet's shapes (WINDOWS windows, default 32) and two
VAE shapes (64 images).  LS_GN_APPLY_V1=1: the grid-stride apply kernel."""
import os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from latentsync_amd import ops


def timeit(f, reps=20):
    f(); torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); f(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts) * 1e3


W = int(os.environ.get('WINDOWS', '32'))
for (n, H, C) in [(16 * W, 32, 320), (16 * W, 16, 640), (16 * W, 8, 1280), (16 * W, 4, 1280), (64, 256, 128), (64, 128, 256)]:
    x = torch.randn(n, H, H, C, device="cuda").to(torch.bfloat16)
    g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    B = n // 16
    t = timeit(lambda: ops.group_norm(x, 32, 1e-5, g, b, B))
    sc, sh = ops.group_norm(x, 32, 1e-5, g, b, B)
    ta = timeit(lambda: ops.group_norm_apply(x, sc, sh, B, True))
    mb = x.numel() * 2 / 1e6
    print(f"v1={os.environ.get('LS_GN_APPLY_V1', '0')} GN {n}x{H}x{H}x{C}: stats {t:7.1f} us ({mb / t:5.2f} TB/s)  "
          f"apply {ta:7.1f} us ({2 * mb / ta:5.2f} TB/s)")
