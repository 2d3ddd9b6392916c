import math, os, sys, collections
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from latentsync_amd import ops, _lib
from latentsync_amd.unet import _Dev
from latentsync_amd.packing import pack_weight

lib = _lib.load()
torch.manual_seed(0)
M, N, C = 512, 960, 320
x = (torch.randn(M, C) * 2 + 3).to(torch.bfloat16).float()
gamma, beta = 1 + 0.1 * torch.randn(C), 0.1 * torch.randn(C)
w = torch.randn(N, C) / math.sqrt(C)
pk = _Dev({}, "cuda").packed_ln(w, None, (gamma, beta))
xd = x.to(torch.bfloat16).cuda()
st = ops.row_stats(xd)
ref = F.layer_norm(x, (C,), gamma, beta, 1e-5) @ w.T
wp = pk.w.float().cpu()[:N, :C]
bias = pk.bias.float().cpu()[:N]
raw = x @ wp.T + bias              # LN not applied to A
zero = bias.expand(M, N)           # acc == 0
for run in range(6):
    y = ops.linear(xd, pk, ln_stats=st).float().cpu()
    e = (y - ref).abs()
    bad = e > 0.05 + 0.05 * ref.abs()
    cnt = collections.Counter()
    kinds = collections.Counter()
    for r, c in bad.nonzero().tolist():
        cnt[(r // 256, (r % 256) // 32, (r % 32) // 16, c // 32)] += 1
        yy = y[r, c]
        k = "raw" if abs(yy - raw[r, c]) < 0.05 + 0.02 * abs(raw[r, c]) else "zero" if abs(yy - zero[r, c]) < 0.02 else "other"
        kinds[k] += 1
    print(f"run{run}: bad {int(bad.sum())} kinds {dict(kinds)} blocks(wg,wave,i,chunk):n {sorted(cnt.items())[:12]}")
