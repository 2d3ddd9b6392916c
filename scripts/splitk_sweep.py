"""Tile x split-K sweep of ls_conv2d on the 4x4-level 3x3 convs (M = 4096 rows at 16
windows per call, N = 1280, K = 11520 / 23040) and the other low-M shapes: which
forced (tile, split) beats the cost model's pick.  usage: python scripts/splitk_sweep.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from latentsync_amd import _lib, ops  # noqa: E402
from latentsync_amd.packing import pack_weight  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import timed  # noqa: E402

lib = _lib.load()
SHAPES = [("conv3x3 1280 @4^2", 256, 4, 1280, 1280, 3), ("conv3x3 2560->1280 @4^2", 256, 4, 2560, 1280, 3),
          ("conv3x3 1280 @8^2", 256, 8, 1280, 1280, 3), ("conv3x3 640 @16^2", 256, 16, 640, 640, 3),
          ("ff2 5120->1280 @4^2", 256, 4, 5120, 1280, 1), ("geglu 1280->10240 @4^2", 256, 4, 1280, 10240, 1)]
TILES = {0: "auto", 9: "128x160", 1: "128x128", 5: "256x256"}

for name, n, H, cin, cout, ks in SHAPES:
    x = torch.randn(n, H, H, cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(cout, cin, ks, ks) / (cin * ks * ks) ** 0.5
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), torch.zeros(cout, device="cuda"), cin, ks, cout)
    fl = 2.0 * n * H * H * cout * cin * ks * ks
    for tile, tname in TILES.items():
        for split in ((1,) if tile == 0 else (1, 2, 3, 4, 6, 8)):
            lib.ls_set_tuning(2, tile)
            lib.ls_set_tuning(3, split if tile else 0)
            try:
                out = ops.conv(x, pw)
                t = timed(lambda: ops.conv(x, pw, out=out))
            except RuntimeError as e:
                print(f"{name:26s} {tname:8s} split {split}: {e}")
                continue
            print(f"{name:26s} {tname:8s} split {split}: {t * 1e3:8.1f} us {fl / t / 1e9:7.1f} TF/s", flush=True)
    lib.ls_set_tuning(2, 0)
    lib.ls_set_tuning(3, 0)
