"""Row-block LayerNorm GEMM run-to-run / vs-fp32 check used in the gfx950 SLP
investigation (scripts/slp_variants.py builds the A/B libraries).
Prints the number of output elements off the fp32 reference (per run, per
(wave-in-block, row-fragment) position) and the run-to-run differing elements.
usage: LS_HIP_LIB=latentsync_amd/libls_hip_<variant>.so python scripts/slp_check.py [runs]"""
import collections
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from latentsync_amd import _lib, ops  # noqa: E402
from latentsync_amd.unet import _Dev  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 16
print("library:", os.environ.get("LS_HIP_LIB", _lib.LIB_PATH), flush=True)
torch.manual_seed(0)
total_bad = total_diff = 0
for M, N, C in ((65536, 960, 320), (16384, 1920, 640), (4096, 960, 320)):
    x = (torch.randn(M, C) * 2 + 3).to(torch.bfloat16).float()
    w = torch.randn(N, C) / math.sqrt(C)
    b = torch.randn(N) * 0.1
    gamma, beta = 1 + 0.1 * torch.randn(C), 0.1 * torch.randn(C)
    xd = x.to(torch.bfloat16).cuda()
    pk = _Dev({}, "cuda").packed_ln(w, b, (gamma, beta))
    st = ops.row_stats(xd)
    ref = (F.layer_norm(x, (C,), gamma, beta, 1e-5) @ w.T + b).cuda()
    first = None
    bad_tot, diff_tot, where = 0, 0, collections.Counter()
    for r in range(runs):
        y = ops.linear(xd, pk, ln_stats=st).float()
        bad = (y - ref).abs() > 0.05 + 0.05 * ref.abs()
        nb = int(bad.sum())
        if nb:
            rows = bad.any(1).nonzero().flatten().cpu()
            where.update(((int(q) % 256) // 32, (int(q) % 32) // 16) for q in rows)
        bad_tot += nb
        if first is None:
            first = y
        else:
            diff_tot += int((y != first).sum())
    print(f"M={M} N={N} C={C}: {runs} runs, elements off the fp32 reference {bad_tot}, "
          f"run-to-run differing {diff_tot}, bad rows by (wave, fragment) {dict(where)}", flush=True)
    total_bad += bad_tot
    total_diff += diff_tot
print(f"TOTAL off-reference {total_bad} run-to-run {total_diff}")
