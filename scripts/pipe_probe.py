"""Deeper operand pipelines on the mid-size GEMMs: auto vs forced tiles 7 (phased
256x256), 8 (4-stage BK 32 256x256), 9 (128x160) and 128x160 with the 4-stage BK 32
ring (ls_set_tuning key 5).  usage: python scripts/pipe_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from latentsync_amd import _lib, ops  # noqa: E402
from latentsync_amd.packing import pack_weight  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import timed  # noqa: E402

lib = _lib.load()
SHAPES = [("ff2 16^2 K2560 N640 res", 65536, 2560, 640, 1, True), ("o-proj 16^2 K640 N640 res", 65536, 640, 640, 1, True),
          ("qkv 8^2 K1280 N3840", 16384, 1280, 3840, 1, False), ("o-proj 8^2 K1280 N1280 res", 16384, 1280, 1280, 1, True),
          ("conv3x3 320 @32^2 res", 262144, 2880, 320, 3, True), ("conv3x3 640 @16^2 res", 65536, 5760, 640, 3, True)]
for name, M, K, N, ks, has_res in SHAPES:
    cin = K // (ks * ks)
    if ks == 1:
        x = torch.randn(1, 1, M, cin, device="cuda").to(torch.bfloat16)
    else:
        H = int(round((M // 256) ** 0.5))
        x = torch.randn(256, H, H, cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, cin, ks, ks) / K ** 0.5
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), torch.zeros(N, device="cuda"), cin, ks, N)
    res = torch.randn(*x.shape[:3], N, device="cuda").to(torch.bfloat16) if has_res else None
    out = ops.conv(x, pw, res=res)
    fl = 2.0 * M * N * K
    for tile, bk, tn in ((0, 64, "auto"), (9, 64, "128x160"), (9, 32, "128x160 BK32x4"), (1, 32, "128x128 BK32x4"),
                         (5, 64, "256x256"), (7, 64, "256x256 phased"), (8, 64, "256x256 BK32x4")):
        lib.ls_set_tuning(2, tile)
        lib.ls_set_tuning(5, bk)
        try:
            t = timed(lambda: ops.conv(x, pw, res=res, out=out))
            print(f"{name:28s} {tn:16s} {t * 1e3:8.1f} us {fl / t / 1e9:7.1f} TF/s", flush=True)
        except RuntimeError as e:
            print(f"{name:28s} {tn:16s} error {e}", flush=True)
    lib.ls_set_tuning(2, 0)
    lib.ls_set_tuning(5, 64)
