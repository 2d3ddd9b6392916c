"""Cost of the GroupNorm column-sum epilogue (ops.conv(gn_out=True)) per tile kernel
on the UNet's 3x3 conv shapes (16 windows per call): with vs without, and the
read-pass alternative (ls_gn_colsum).  usage: python scripts/gn_epilogue_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from latentsync_amd import _lib, ops  # noqa: E402
from latentsync_amd.packing import pack_weight  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import timed  # noqa: E402

lib = _lib.load()
SHAPES = [("conv3x3 320 @32^2", 256, 32, 320, 320), ("conv3x3 640 @16^2", 256, 16, 640, 640),
          ("conv3x3 1280 @8^2", 256, 8, 1280, 1280), ("conv3x3 1920->640 @16^2", 256, 16, 1920, 640),
          ("vae 128 @256^2", 32, 256, 128, 128), ("vae 256 @128^2", 32, 128, 256, 256)]
for name, n, H, cin, cout in SHAPES:
    x = torch.randn(n, H, H, cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    pw = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), torch.zeros(cout, device="cuda"), cin, 3, cout)
    res = torch.randn(n, H, H, cout, device="cuda").to(torch.bfloat16)
    out = ops.conv(x, pw, res=res)
    t0 = timed(lambda: ops.conv(x, pw, res=res, out=out))
    t1 = timed(lambda: ops.conv(x, pw, res=res, out=out, gn_out=True))
    t2 = timed(lambda: ops.gn_colsum(out))
    print(f"{name:26s} plain {t0 * 1e3:8.1f} us  +epilogue sums {t1 * 1e3:8.1f} us ({(t1 / t0 - 1) * 100:+.1f} %)"
          f"  read pass {t2 * 1e3:7.1f} us", flush=True)
