"""bf16-storage emulation of the fp32 oracle (TEST INFRASTRUCTURE ONLY -- imported by tests/,
never by the product path).

The HIP path stores weights and every op's output in bf16 and accumulates in fp32; the
oracle (oracle/ref_cpu.py) runs fp32 end to end.  `bf16_storage()` rounds the output of each
torch op the oracle's layers are built from (conv2d, linear, group_norm, layer_norm, silu,
gelu, scaled_dot_product_attention, interpolate) to bf16, and `bf16_weights(sd)` rounds a
state dict -- an independent bf16 implementation of the same algorithm, whose distance from
the fp32 oracle is the deviation bf16 storage alone produces.  It is the yardstick for the
GPU's per-pixel deviation (tests/test_serve_gpu.py): the GPU rounds at other points (fused
epilogues, fp32 DDIM state), so the two do not agree bit for bit, but a GPU deviation far
beyond the emulated one would be a defect, not rounding."""
import contextlib

import torch
import torch.nn.functional as F

OPS = ("conv2d", "linear", "group_norm", "layer_norm", "silu", "gelu", "scaled_dot_product_attention", "interpolate")


def bf16_weights(sd):
    return {k: v.to(torch.bfloat16).float() if torch.is_tensor(v) and v.is_floating_point() else v
            for k, v in sd.items()}


@contextlib.contextmanager
def bf16_storage():
    orig = {n: getattr(F, n) for n in OPS}

    def wrap(fn):
        def f(*a, **k):
            y = fn(*a, **k)
            return y.to(torch.bfloat16).float() if y.is_floating_point() else y
        return f
    try:
        for n, fn in orig.items():
            setattr(F, n, wrap(fn))
        yield
    finally:
        for n, fn in orig.items():
            setattr(F, n, fn)
