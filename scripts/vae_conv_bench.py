"""VAE 256x256 128-channel 3x3 conv: materialised GN-apply+SiLU then the DMA conv,
vs the register-staged conv with the GN affine+SiLU fused into its A loads,
vs forced tiles.  (16 frames x 8 windows.)"""
import os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from latentsync_amd import ops, _lib
from latentsync_amd.packing import pack_weight

lib = _lib.load()


def timeit(f, reps=10):
    f(); torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); f(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts) * 1e3


for n, H, C, N in [(128, 256, 128, 128), (128, 128, 256, 256), (128, 64, 512, 512)]:
    x = torch.randn(n, H, H, C, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, C, 3, 3) / (9 * C) ** 0.5
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), torch.zeros(N, device="cuda"), C, 3, N)
    g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    S = n  # VAE GroupNorm: per-image statistics
    sc, sh = ops.group_norm(x, 32, 1e-6, g, b, S)
    out = torch.empty(n, H, H, N, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * n * H * H * N * C * 9
    t_app = timeit(lambda: ops.group_norm_apply(x, sc, sh, S, True))
    a = ops.group_norm_apply(x, sc, sh, S, True)
    t_conv = timeit(lambda: ops.conv(a, pw, out=out))
    t_fused = timeit(lambda: ops.conv(x, pw, aff=(sc, sh, 1, True), out=out))
    line = f"{n}x{H}x{H}x{C}->{N}: apply {t_app:7.0f} + conv {t_conv:7.0f} = {t_app + t_conv:7.0f} us | fused(regstage) {t_fused:7.0f} us"
    for tile in (1, 6, 5):
        lib.ls_set_tuning(2, tile)
        try:
            t = timeit(lambda: ops.conv(a, pw, out=out))
            line += f" | t{tile} {t:7.0f}"
        except Exception as e:  # noqa: BLE001
            line += f" | t{tile} err"
        lib.ls_set_tuning(2, 0)
    print(line + f"  ({fl / t_conv / 1e6:.0f} TF/s dma)", flush=True)
