"""Where the time of the short-K / residual GEMMs goes (the UNet's o-proj / proj_out /
small linears): each shape timed with the kernel's ablation switches (ls_set_tuning
key 4: 2 = no operand DMA, 4 = no epilogue stores, 16 = no MFMAs), plus the tile
forced to the alternatives.  usage: python scripts/small_gemm_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from latentsync_amd import _lib, ops  # noqa: E402
from latentsync_amd.packing import pack_weight  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import timed  # noqa: E402

lib = _lib.load()
SHAPES = [("o-proj 16^2 K640 N640 res", 65536, 640, 640, True), ("o-proj 8^2 K1280 N1280 res", 16384, 1280, 1280, True),
          ("proj 8^2 K1280 N1280", 16384, 1280, 1280, False), ("o-proj 32^2 K320 N320 res", 262144, 320, 320, True),
          ("ff2 16^2 K2560 N640 res", 65536, 2560, 640, True)]
TILES = {0: "auto", 9: "128x160", 1: "128x128", 5: "256x256", 3: "64x64"}
for name, M, K, N, has_res in SHAPES:
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K) / K ** 0.5
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), torch.zeros(N, device="cuda"), K, 1, N)
    res = torch.randn(M, N, device="cuda").to(torch.bfloat16) if has_res else None
    fl = 2.0 * M * N * K
    by = 2.0 * (M * K + M * N * (2 if has_res else 1))
    out = ops.linear(x, pw, res=res)
    for tile, tn in TILES.items():
        for abl in ((0, 2, 4, 16, 18) if tile in (0, 9) else (0,)):
            lib.ls_set_tuning(2, tile)
            lib.ls_set_tuning(4, abl)
            t = timed(lambda: ops.linear(x, pw, res=res, out=out))
            lib.ls_set_tuning(4, 0)
            print(f"{name:28s} {tn:8s} ablate {abl:2d}: {t * 1e3:8.1f} us  {fl / t / 1e9:7.1f} TF/s  "
                  f"{by / t / 1e9:7.1f} GB/s (algorithmic bytes)", flush=True)
    lib.ls_set_tuning(2, 0)
