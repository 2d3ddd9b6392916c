"""LipsyncPipeline.run_windows across ranks on CPU (gloo, world size 2 and 3): the
window loop's sharding and its exchange, with the window compute replaced by a
deterministic stand-in engine (the compute itself is pinned by the GPU tests).

Checks: ONE collective per clip -- a single all-gather of the fp32
pasted frames, the uint8 frames derived from it -- and every rank's result equal to
the single-process result, short last window included."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from latentsync_amd.pipeline import LipsyncPipeline, frames_to_u8

R, FR = 16, 4


class _Cfg(dict):
    __getattr__ = dict.__getitem__


class _Stub:
    def __init__(self, **kw):
        self.config = _Cfg(kw)
        self.device = torch.device("cpu")


class _Engine:
    """Stand-in WindowEngine: the 'decoded' frames are a fixed function of the
    window's own faces, audio and VAE noise (as the real window is)."""

    def __init__(self, frames, windows):
        self.F, self.nw = frames, windows

    def load(self, faces, mask, audio, init, em, er):
        v = faces.float() / 127.5 - 1 + 0.01 * audio.mean((1, 2))[:, None, None, None] + \
            0.01 * em.mean((1, 2, 3))[:, None, None, None] - 0.01 * er.mean((1, 2, 3))[:, None, None, None]
        self.out = v.clamp(-1, 1) * mask
        self.out_u8 = frames_to_u8(self.out)

    def run(self, callback=None, callback_steps=1):
        return self.out


def _pipe():
    sched = _Stub(steps_offset=1, clip_sample=False)
    sched.init_noise_sigma = 1.0
    pipe = LipsyncPipeline(_Stub(block_out_channels=(8, 8, 8, 8), latent_channels=4), None, _Stub(), sched)
    pipe.engine = lambda Fw, R_, steps, g, use_graphs=True, windows=1: _Engine(Fw, windows)
    pipe.windows_per_batch = 2
    return pipe


def _inputs(n):
    g = torch.Generator().manual_seed(3)
    faces = (torch.rand((n, 3, R, R), generator=g) * 255).to(torch.uint8)
    chunks = torch.randn((n, 50, 384), generator=g)
    mask = (torch.rand((R, R), generator=g) > 0.3).float()
    return faces, chunks, mask


def _run(pipe, n):
    faces, chunks, mask = _inputs(n)
    return pipe.run_windows(faces, chunks, mask, num_frames=FR, num_inference_steps=2, guidance_scale=1.0,
                            generator=torch.Generator().manual_seed(11))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []
    for name in ("all_gather", "all_gather_into_tensor", "all_reduce", "broadcast", "gather", "all_to_all"):
        real = getattr(dist, name)

        def counted(*a, _real=real, _name=name, **k):
            calls.append(_name)
            return _real(*a, **k)
        setattr(dist, name, counted)
    try:
        out, out8 = _run(_pipe(), n)
        # by value (numpy), not torch's fd-shared storage: this process may exit before
        # the parent unpickles, and the storage's fd listener goes with it
        q.put((rank, calls, out.numpy(), out8.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 4 * FR), (3, 5 * FR + 2)])
def test_run_windows_one_collective(world, n):
    ref, ref8 = _run(_pipe(), n)  # single process
    assert ref.shape == (n, 3, R, R) and ref8.shape == (n, R, R, 3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, calls, out, out8 in res:
        assert calls == ["all_gather"], (rank, calls)  # gloo's form of all_gather_into_tensor
        assert torch.equal(torch.from_numpy(out), ref) and torch.equal(torch.from_numpy(out8), ref8), rank


def test_frames_to_u8_matches_paste_back_rounding():
    v = torch.tensor([-1.5, -1.0, -0.999, 0.0, 0.00392, 0.5, 0.99, 1.0, 2.0]).view(1, 1, 3, 3).expand(1, 3, 3, 3)
    u = frames_to_u8(v.contiguous())
    want = [int(min(max(x / 2 + 0.5, 0.0), 1.0) * 255) for x in v[0, 0].flatten().tolist()]
    assert u[0, ..., 0].flatten().tolist() == want
