"""The GELU the GEGLU epilogues and FeedForward kernels evaluate (ls_common.h gelu_erf:
x * sigmoid(x (a + b x^2 + c x^4)), x^2 clamped at 36, log2(e) and the sign folded into the
coefficients) against the exact erf GELU of diffusers' GEGLU (F.gelu, approximate="none").
The coefficients are read from the kernel source, evaluated in float32 the way the kernel does
(fma order, v_exp_f32 = 2^x), and must stay within the 2.6e-5 the source claims."""
import os
import re

import numpy as np
from scipy.special import erf

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "latentsync_amd", "csrc",
                   "ls_common.h")


def _coeffs():
    body = open(SRC).read()
    body = body[body.index("float gelu_erf(float x)"):]
    body = body[:body.index("}")]
    clamp = float(re.search(r"fminf\(x \* x, ([0-9.]+)f\)", body).group(1))
    c, b, a = (float(v) for v in re.search(r"fmaf\(x2, fmaf\(x2, ([-0-9.e]+)f, ([-0-9.e]+)f\), ([-0-9.e]+)f\)",
                                           body).groups())
    return clamp, a, b, c


def test_gelu_form_matches_erf_gelu():
    clamp, a, b, c = _coeffs()
    x = np.linspace(-30, 30, 600001).astype(np.float32)
    x2 = np.minimum(x * x, np.float32(clamp))
    t = (np.float32(c) * x2 + np.float32(b)) * x2 + np.float32(a)
    with np.errstate(over="ignore"):
        y = x / (np.float32(1) + np.exp2(x * t))
    xd = x.astype(np.float64)
    exact = 0.5 * xd * (1 + erf(xd / np.sqrt(2)))
    err = np.abs(y.astype(np.float64) - exact)
    assert err.max() < 2.7e-5, err.max()
    # the tails: gelu(x) -> x for large x, -> -0 for very negative x (2^(x t) overflows to inf)
    assert abs(float(y[-1]) - 30.0) < 1e-5 and abs(float(y[0])) < 1e-6
