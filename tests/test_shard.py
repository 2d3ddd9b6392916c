"""Window sharding + the single all-gather on CPU with gloo,
world_size 2 (and 3 for a ragged split).  The same code runs over RCCL in
bench.py / LipsyncPipeline.run_windows."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from latentsync_amd.shard import gather_windows, rank_windows


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_windows, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = rank_windows(n_windows, world, rank)
        # a "decoded window": (F=4, 8, 8, 3) uint8 frames stamped with the window index
        local = torch.stack([torch.full((4, 8, 8, 3), w, dtype=torch.uint8) for w in mine]) if mine else \
            torch.empty((0, 4, 8, 8, 3), dtype=torch.uint8)
        out = gather_windows(local, n_windows)
        q.put((rank, out[:, 0, 0, 0, 0].tolist(), tuple(out.shape)))
    finally:
        dist.destroy_process_group()


def _run(world, n_windows):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_windows, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_rank_windows_partition():
    for world in (1, 2, 3, 8):
        for n in (0, 1, 5, 16, 17):
            got = sorted(i for r in range(world) for i in rank_windows(n, world, r))
            assert got == list(range(n))
    with pytest.raises(ValueError):
        rank_windows(4, 2, 2)


@pytest.mark.parametrize("world,n_windows", [(2, 4), (2, 5), (3, 7)])
def test_gather_windows_clip_order(world, n_windows):
    for rank, order, shape in _run(world, n_windows):
        assert order == list(range(n_windows)), (rank, order)
        assert shape == (n_windows, 4, 8, 8, 3)


def test_gather_single_process_is_identity():
    x = torch.arange(6, dtype=torch.uint8).view(3, 2)
    assert gather_windows(x, 3) is x
    with pytest.raises(ValueError):
        gather_windows(x, 4)
