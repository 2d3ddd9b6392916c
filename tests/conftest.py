import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long CPU test (full-size UNet oracle)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def block_sd(prefix, shapes, seed):
    """State dict for a stand-alone block: keys drawn WITHOUT the prefix (as the
    reference module's own named_parameters), stored under ``prefix.key``."""
    import torch
    from latentsync_amd.weights import init_tensor, is_buffer_key
    return {f"{prefix}.{k}": init_tensor(k, s, seed) for k, s in shapes.items() if not is_buffer_key(k)}


def rel_err(a, b):
    import torch
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.fixture
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
