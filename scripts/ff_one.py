"""Launch the fused C = 320 FeedForward (ls_feedforward) repeatedly at the 32x32 level of a
48-window UNet call (M = 786432 rows): a PMC / trace target, HIP-event time printed.
usage: python scripts/ff_one.py [reps]"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from latentsync_amd import ops  # noqa: E402
from latentsync_amd.packing import pack_ff_w2  # noqa: E402
from latentsync_amd.unet import _Dev  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
M, C, I = int(os.environ.get("FF_M", 786432)), 320, 1280
g = torch.Generator().manual_seed(0)
r = lambda *s, sc=1.0: torch.randn(s, generator=g) * sc
dv = _Dev({"w2": r(C, I, sc=1 / math.sqrt(I)), "b2": r(C, sc=0.1)}, "cuda")
ff1 = dv.packed_ln(r(2 * I, C, sc=1 / math.sqrt(C)), r(2 * I, sc=0.1), (1 + 0.2 * r(C), 0.1 * r(C)), geglu=True)
ff2 = dv.packed("w2", "b2")
ff2p = pack_ff_w2(dv.sd["w2"].float()).to(torch.bfloat16).cuda()
x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
st = ops.row_stats(x)
y = ops.feedforward(x, st, ff1, ff2, ff2p)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    ops.feedforward(x, st, ff1, ff2, ff2p, out=y)
e1.record()
torch.cuda.synchronize()
t = e0.elapsed_time(e1) / reps
fl = 2.0 * M * 2 * I * C + 2.0 * M * C * I
print(f"ff_fused M={M}: {t * 1e3:.1f} us  {fl / t / 1e9:.1f} TF/s")
