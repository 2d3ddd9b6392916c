import math, os, sys, collections
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from latentsync_amd import ops, _lib
from latentsync_amd.unet import _Dev
from latentsync_amd.packing import pack_weight

lib = _lib.load()
torch.manual_seed(0)
M, N, C = 4096, 960, 320
x = (torch.randn(M, C) * 2 + 3).to(torch.bfloat16).float()
w = torch.randn(N, C) / math.sqrt(C)
b = torch.randn(N) * 0.1
xd = x.to(torch.bfloat16).cuda()
res = torch.randn(M, N).to(torch.bfloat16)
for case in ["plain", "res", "ln"]:
    kw = {}
    if case == "ln":
        gamma, beta = 1 + 0.1 * torch.randn(C), 0.1 * torch.randn(C)
        pk = _Dev({}, "cuda").packed_ln(w, b, (gamma, beta))
        kw["ln_stats"] = ops.row_stats(xd)
        ref = F.layer_norm(x, (C,), gamma, beta, 1e-5) @ w.T + b
    else:
        pk = ops.Packed(pack_weight(w).to(torch.bfloat16).cuda(), b.cuda(), C, 1, N)
        ref = x @ pk.w.float().cpu()[:, :C].T + b
        if case == "res":
            kw["res"] = res.cuda()
            ref = ref + res.float()
    tot = 0
    for run in range(8):
        y = ops.linear(xd, pk, **kw).float().cpu()
        bad = (y - ref).abs() > 0.05 + 0.05 * ref.abs()
        cnt = collections.Counter(((r % 256) // 32, (r % 32) // 16) for r, c in bad.nonzero().tolist())
        tot += int(bad.sum())
        if bad.any():
            print(f"{case} run{run}: bad {int(bad.sum())} (wave,i): {dict(cnt)}")
    print(f"{case}: total bad {tot}")

if os.environ.get("LS_RB_DEBUG"):
    from latentsync_amd.ops import workspace
    gamma, beta = 1 + 0.1 * torch.randn(C), 0.1 * torch.randn(C)
    pk = _Dev({}, "cuda").packed_ln(w, b, (gamma, beta))
    st = ops.row_stats(xd)
    ws = workspace(xd.device)
    for run in range(6):
        ws.gemm.zero_()
        y = ops.linear(xd, pk, ln_stats=st)
        torch.cuda.synchronize()
        seen = ws.gemm[: M * 8].view(torch.float32).view(M, 2).cpu()
        ok = (seen == st.view(M, 2).cpu()).all(1)
        badr = (~ok).nonzero().flatten()
        print(f"stats seen by kernel run{run}: wrong rows {len(badr)} {badr[:10].tolist()} "
              f"e.g. seen {seen[badr[:2]].tolist()} true {st.view(M, 2).cpu()[badr[:2]].tolist()}")
