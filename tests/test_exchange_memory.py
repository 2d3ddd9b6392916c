"""configs[3] memory: the bench's end-of-loop exchange at 8 ranks fits one MI355X.

bench.py at `--gpus 8 --steps 20` (48 windows per batch, 256^2) keeps each rank's
960 windows of fp32 pasted frames, all-gathers every rank's frames once into a receive
buffer that is already clip order (shard.gather_windows, no reordering copy) and derives
the uint8 clip from it in bounded chunks (pipeline.frames_to_u8).  This computes that
footprint and checks it beside the engine footprint MEASURED on the MI355X
(profiles/r06a_bench.json, `memory.engine_gb` = torch.cuda.max_memory_allocated after
the engine's capture and warm-up), with margin against the card's HBM."""
import json
import os

import pytest
import torch

import bench
from latentsync_amd import shard
from latentsync_amd.pipeline import U8_CHUNK, frames_to_u8

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GIB = 1024 ** 3


def _measured():
    with open(os.path.join(REPO, "profiles", "r06a_bench.json")) as f:
        return json.load(f)["memory"]


def test_exchange_bytes_formula():
    win32 = 16 * 3 * 256 * 256 * 4
    n = 8 * 20 * 48
    want = 20 * 48 * win32 + 8 * 20 * 48 * win32 + n * 16 * 256 * 256 * 3 + 2 * U8_CHUNK * 3 * 256 * 256 * 4
    assert bench.exchange_bytes(8, 20, 48) == want
    # world 1: no receive buffer, the rank's own frames are the clip
    assert bench.exchange_bytes(1, 20, 48) == 20 * 48 * win32 + 20 * 48 * 16 * 256 * 256 * 3 + \
        2 * U8_CHUNK * 3 * 256 * 256 * 4
    assert shard.gather_bytes(7, 3, 10) == 4 * 3 * 10  # receive 3 x 3 slabs + one padded send slab


def test_8_rank_footprint_fits_hbm():
    m = _measured()
    ex = bench.exchange_bytes(8, 20, 48) / GIB
    total = m["engine_gb"] + ex
    print(f"per-rank at 8 ranks, --steps 20: engine {m['engine_gb']:.1f} + exchange {ex:.1f} = {total:.1f} GiB "
          f"of {m['hbm_total_gb']:.0f}")
    assert total < 0.8 * m["hbm_total_gb"]
    # the round-5 exchange (fp32 gather + index_select copy + two full-size frames_to_u8
    # temporaries) would not have fit: >= 290 GB beside the engine
    win32 = 16 * 3 * 256 * 256 * 4
    old = (20 * 48 + 4 * 8 * 20 * 48) * win32 / GIB
    assert m["engine_gb"] + old > m["hbm_total_gb"]


def test_frames_to_u8_chunked_matches_whole():
    g = torch.Generator().manual_seed(0)
    x = torch.rand((2 * U8_CHUNK + 3, 3, 4, 5), generator=g) * 2.4 - 1.2
    whole = ((x / 2 + 0.5).clamp(0, 1) * 255).to(torch.uint8).permute(0, 2, 3, 1)
    assert torch.equal(frames_to_u8(x), whole)
