"""Weight packing K order (include/ls_hip.h ls_conv2d, latentsync_amd/packing.py): the
column k of a packed [N][K] weight must hold the (tap, input channel) the kernels' gather
reads for that k.  CPU-only: checks the layout against the index formula."""
import pytest
import torch

from latentsync_amd import packing


def _unpack_index(O, I, kind):
    """k -> (tap, ci) as ls_conv2d reads it."""
    idx = []
    for k in range(9 * I):
        if kind == "ccm":  # ABI 10: channel-chunk-major, taps innermost
            chunk, rem = divmod(k, 576)
            idx.append((rem // 64, chunk * 64 + rem % 64))
        else:  # tap-major
            idx.append((k // I, k % I))
    return idx


@pytest.mark.parametrize("I,kind", [(64, "ccm"), (320, "ccm"), (128, "ccm"), (24, "tap"), (80, "tap")])
def test_pack3x3_order(I, kind):
    O = 3
    w = torch.arange(O * I * 9, dtype=torch.float32).reshape(O, I, 3, 3)
    p = packing.pack_weight(w)
    for k, (tap, ci) in enumerate(_unpack_index(O, I, kind)):
        kh, kw = divmod(tap, 3)
        assert torch.equal(p[:, k], w[:, ci, kh, kw]), (k, tap, ci)
    assert p.shape[1] % 64 == 0 and torch.all(p[:, 9 * I:] == 0)


def test_pack1x1_unchanged():
    w = torch.randn(5, 320)
    assert torch.equal(packing.pack_weight(w)[:, :320], w)
