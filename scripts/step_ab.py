"""Time one denoising step (UNet fwd + CFG/DDIM, graph-replayed) of the bench
workload -- for A/B builds: LS_HIP_LIB=path/to/other.so python scripts/step_ab.py
usage: python scripts/step_ab.py [windows] [resolution]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from latentsync_amd.config import STAGE2_MODEL  # noqa: E402
from latentsync_amd.pipeline import WindowEngine, load_fixed_mask  # noqa: E402
from latentsync_amd.scheduler import DDIMScheduler  # noqa: E402
from latentsync_amd.unet import UNet3DConditionModel  # noqa: E402
from latentsync_amd.vae import AutoencoderKL  # noqa: E402

nw = int(sys.argv[1]) if len(sys.argv) > 1 else 8
R = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dev = torch.device("cuda", 0)
unet = UNet3DConditionModel(**STAGE2_MODEL).init_weights(41).to(dev).eval()
vae = AutoencoderKL().init_weights(51).to(dev)
eng = WindowEngine(unet, vae, DDIMScheduler(**bench.SCHED_CFG), 16, R, 20, 1.0, windows=nw)
eng.load(*bench.synthetic_window(16 * nw, R, R // 8, 384, 1000, dev)[:1], load_fixed_mask(R).to(dev),
         *bench.synthetic_window(16 * nw, R, R // 8, 384, 1000, dev)[1:])
eng.capture()
g_enc, g_step, g_dec = eng.graphs
for _ in range(3):
    g_step.replay()
torch.cuda.synchronize()
ts = []
for _ in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g_step.replay()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ts.sort()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); g_enc.replay(); e1.record(); torch.cuda.synchronize(); te = e0.elapsed_time(e1)
e0.record(); g_dec.replay(); e1.record(); torch.cuda.synchronize(); td = e0.elapsed_time(e1)
print(f"{os.environ.get('LS_HIP_LIB', 'default')}: windows {nw} R {R}: step median {ts[5]:.3f} ms "
      f"(min {ts[0]:.3f}), encode {te:.2f} ms, decode {td:.2f} ms")
