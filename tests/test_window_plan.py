"""Engine-size planning of LipsyncPipeline.run_windows (pipeline.plan_window_batches):
clips of different lengths share captured engines, every window runs exactly once, no
engine exceeds windows_per_batch, and padding stays below one bucket step.  CPU only."""
import math

import pytest

from latentsync_amd.pipeline import WINDOW_BUCKETS, plan_window_batches


def test_neighbouring_lengths_share_an_engine():
    e10, b10 = plan_window_batches(list(range(10)), 48)
    e11, b11 = plan_window_batches(list(range(11)), 48)
    assert e10 == e11 == 16 and b10 == [list(range(10))] and b11 == [list(range(11))]


@pytest.mark.parametrize("cap", [1, 2, 16, 32, 48, 40, 5])
def test_plan_covers_every_window_once(cap):
    for n in range(0, 150):
        full = [3 * i + 1 for i in range(n)]  # rank-local indices need not be contiguous
        E, batches = plan_window_batches(full, cap)
        if n == 0:
            assert (E, batches) == (0, [])
            continue
        assert [i for b in batches for i in b] == full
        assert 1 <= E <= cap and (E in WINDOW_BUCKETS or E == cap)
        assert all(len(b) == E for b in batches[:-1]) and 1 <= len(batches[-1]) <= E
        # no more engine passes than the old equal split, and the padded work is bounded
        assert len(batches) == math.ceil(n / cap) or len(batches) == math.ceil(n / E)
        assert len(batches) <= math.ceil(n / cap) + 1
        padded = E * len(batches) - n
        steps = sorted({b for b in WINDOW_BUCKETS if b < cap} | {cap})
        gap = max(b - a for a, b in zip([0] + steps, steps))
        assert padded < gap * len(batches)


def test_engine_sizes_are_few():
    """Every clip length up to 200 windows maps to one of at most len(WINDOW_BUCKETS) engines."""
    sizes = {plan_window_batches(list(range(n)), 48)[0] for n in range(1, 201)}
    assert sizes <= set(WINDOW_BUCKETS)
