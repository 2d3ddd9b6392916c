"""Two window batches in flight on two HIP streams: is there idle GPU time (kernel tails,
small grids, launch gaps) that a second independent batch fills?  Times K full window
batches (encode graph, 20 step graphs, decode graph) of two 48-window engines run back to
back on one stream against the same batches run concurrently on two streams.
usage: python scripts/concurrency_probe.py [windows] [K]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from latentsync_amd.config import STAGE2_MODEL  # noqa: E402
from latentsync_amd.pipeline import WindowEngine, load_fixed_mask  # noqa: E402
from latentsync_amd.scheduler import DDIMScheduler  # noqa: E402
from latentsync_amd.unet import UNet3DConditionModel  # noqa: E402
from latentsync_amd.vae import AutoencoderKL  # noqa: E402

nw = int(sys.argv[1]) if len(sys.argv) > 1 else 48
K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
R = 256
dev = torch.device("cuda", 0)
unet = UNet3DConditionModel(**STAGE2_MODEL).init_weights(41).to(dev).eval()
vae = AutoencoderKL().init_weights(51).to(dev)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
engs = []
for i in range(2):
    e = WindowEngine(unet, vae, DDIMScheduler(**bench.SCHED_CFG), 16, R, 20, 1.0, windows=nw)
    inp = bench.synthetic_window(16 * nw, R, R // 8, 384, 1000 + i, dev)
    e.load(inp[0], load_fixed_mask(R).to(dev), *inp[1:])
    e.capture()
    engs.append(e)
torch.cuda.synchronize()


def run(e):
    g_enc, g_step, g_dec = e.graphs
    g_enc.replay()
    for _ in range(e.steps):
        g_step.replay()
    g_dec.replay()


def timed(fn):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    for s in streams:
        torch.cuda.current_stream().wait_stream(s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def serial():
    for _ in range(K):
        run(engs[0])
        run(engs[1])


def concurrent():
    cur = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(cur)
    for _ in range(K):
        for e, s in zip(engs, streams):
            with torch.cuda.stream(s):
                run(e)


serial()
concurrent()
for r in range(3):
    ts, tc = timed(serial), timed(concurrent)
    fr = 2 * K * nw * 16
    print(f"round {r}: {2 * K} batches of {nw} windows: one stream {ts:.1f} ms ({fr / ts * 1e3:.1f} frames/s), "
          f"two streams {tc:.1f} ms ({fr / tc * 1e3:.1f} frames/s), ratio {tc / ts:.3f}", flush=True)
