"""256x256 tile kernels (big = 5, phased = 7, 4-stage = 8) on square GEMMs and UNet
shapes.  usage: python scripts/p8_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from latentsync_amd import _lib, ops  # noqa: E402
from latentsync_amd.packing import pack_weight  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import timed  # noqa: E402

lib = _lib.load()
SHAPES = [("square 8192", 8192, 8192, 8192, 1, False), ("square 4096", 4096, 4096, 4096, 1, False),
          ("ff2 16^2 K2560 N640 res", 65536, 2560, 640, 1, True), ("qkv 8^2 K1280 N3840", 16384, 1280, 3840, 1, False),
          ("geglu 8^2 K1280 N10240", 16384, 1280, 10240, 1, False),
          ("conv3x3 640 @16^2 res", 65536, 5760, 640, 3, True), ("conv3x3 1280 @8^2 res", 16384, 11520, 1280, 3, True),
          ("vae 512 @64^2", 131072, 4608, 512, 3, False)]
for name, M, K, N, ks, has_res in SHAPES:
    cin = K // (ks * ks)
    if ks == 1:
        x = (torch.rand(1, 1, M, cin, device="cuda") * 2 - 1).to(torch.bfloat16)
    else:
        n = 32 if name.startswith("vae") else 256
        H = int(round((M // n) ** 0.5))
        x = (torch.rand(n, H, H, cin, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, cin, ks, ks) * 2 - 1) / K ** 0.5
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), torch.zeros(N, device="cuda"), cin, ks, N)
    res = torch.randn(*x.shape[:3], N, device="cuda").to(torch.bfloat16) if has_res else None
    out = ops.conv(x, pw, res=res)
    ref = out.float().clone()
    fl = 2.0 * M * N * K
    for tile, tn in ((0, "auto"), (5, "256x256"), (7, "256x256 phased"), (9, "128x160")):
        lib.ls_set_tuning(2, tile)
        t = timed(lambda: ops.conv(x, pw, res=res, out=out))
        err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
        print(f"{name:26s} {tn:16s} {t * 1e3:8.1f} us {fl / t / 1e9:7.1f} TF/s  max rel diff vs auto {err:.2e}",
              flush=True)
    lib.ls_set_tuning(2, 0)
