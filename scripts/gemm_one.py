"""Launch one ls_conv2d shape repeatedly (PMC / trace target).
env: SHAPE="M K N ks res" (default the 16x16-level ff2: 65536 2560 640 1 1), TILE (forced
tile id, 0 = auto), REPS (20), AFF=1 (GroupNorm affine on a 3x3 input).  usage: python scripts/gemm_one.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from latentsync_amd import _lib, ops  # noqa: E402
from latentsync_amd.packing import pack_weight  # noqa: E402

M, K, N, ks, has_res = (int(v) for v in os.environ.get("SHAPE", "65536 2560 640 1 1").split())
lib = _lib.load()
lib.ls_set_tuning(2, int(os.environ.get("TILE", "0")))
if ks == 1:
    x = torch.randn(1, 1, M, K, device="cuda").to(torch.bfloat16)
else:  # 3x3 on 16 frames of a square image with M / 16 pixels... (H = W = sqrt(M / n))
    n = 256
    H = int(round((M // n) ** 0.5))
    x = torch.randn(n, H, H, K // 9, device="cuda").to(torch.bfloat16)
cin = K // (ks * ks)
w = torch.randn(N, cin, ks, ks) / K ** 0.5
pw = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), torch.zeros(N, device="cuda"), cin, ks, N)
res = torch.randn(*x.shape[:3], N, device="cuda").to(torch.bfloat16) if has_res else None
kw = {}
if os.environ.get("AFF") and ks == 3:  # GroupNorm affine + SiLU on the input (the halo conv's GN variant)
    kw = dict(aff=(torch.rand(x.shape[0], cin, device="cuda") + 0.5, torch.randn(x.shape[0], cin, device="cuda") * 0.1, 1, True),
              aff_materialize=True)
out = ops.conv(x, pw, res=res, **kw)
for _ in range(int(os.environ.get("REPS", "20"))):
    ops.conv(x, pw, res=res, out=out, **kw)
torch.cuda.synchronize()
print("done", M, K, N, ks, has_res)
