"""Engine-size planning of LipsyncPipeline.run_windows (pipeline.plan_window_batches):
clips of different lengths share captured engines, every window runs exactly once, no
engine exceeds windows_per_batch, and padding stays within MAX_PAD of the clip (or
under one window per batch when the engine is sized exactly).  CPU only."""
import math

import pytest

from latentsync_amd.pipeline import MAX_PAD, WINDOW_BUCKETS, plan_window_batches


def test_neighbouring_lengths_share_an_engine():
    e10, b10 = plan_window_batches(list(range(10)), 48)
    e11, b11 = plan_window_batches(list(range(11)), 48)
    assert e10 == e11 == 12 and b10 == [list(range(10))] and b11 == [list(range(11))]


@pytest.mark.parametrize("cap", [1, 2, 16, 32, 48, 40, 5])
def test_plan_covers_every_window_once(cap):
    for n in range(0, 150):
        full = [3 * i + 1 for i in range(n)]  # rank-local indices need not be contiguous
        E, batches = plan_window_batches(full, cap)
        if n == 0:
            assert (E, batches) == (0, [])
            continue
        assert [i for b in batches for i in b] == full
        per = math.ceil(n / math.ceil(n / cap))
        assert 1 <= E <= cap and (E in WINDOW_BUCKETS or E in (cap, per))
        assert all(len(b) == E for b in batches[:-1]) and 1 <= len(batches[-1]) <= E
        # never more engine passes than the equal split into ceil(n / cap) batches
        assert len(batches) <= math.ceil(n / cap)
        padded = E * len(batches) - n
        assert padded <= max(MAX_PAD * n, len(batches) - 1), (n, cap, E, padded)


def test_unlucky_lengths_pad_little():
    """49 windows had run as 2 x 32 (+31 %), 9 as 16 (+78 %), 5 as 8 (+60 %)."""
    assert plan_window_batches(list(range(49)), 48)[0] == 28   # 56 windows, +14 %
    assert plan_window_batches(list(range(9)), 48)[0] == 9     # exact
    assert plan_window_batches(list(range(5)), 48)[0] == 6     # +20 %
    assert plan_window_batches(list(range(25)), 48)[0] == 28   # +12 %


def test_engine_sizes_are_few():
    """Clip lengths up to 200 windows map to the buckets plus a few exact sizes."""
    sizes = {plan_window_batches(list(range(n)), 48)[0] for n in range(1, 201)}
    print(sorted(sizes))
    assert len(sizes - set(WINDOW_BUCKETS)) <= 12
