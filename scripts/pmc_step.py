"""Eager (no hipGraph) denoising steps of the bench workload, for rocprofv3 --pmc
passes (counter collection serialises dispatches; graphs are not needed here).
usage: python scripts/pmc_step.py [windows] [steps]"""
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

nw = int(sys.argv[1]) if len(sys.argv) > 1 else 8
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
unet = UNet3DConditionModel(**STAGE2_MODEL).init_weights(41).to(dev).eval()
vae = AutoencoderKL().init_weights(51).to(dev)
eng = WindowEngine(unet, vae, DDIMScheduler(**bench.SCHED_CFG), 16, 256, 20, 1.0, use_graphs=False, windows=nw)
faces, audio, init, em, er = bench.synthetic_window(16 * nw, 256, 32, 384, 1000, dev)
eng.load(faces, load_fixed_mask(256).to(dev), audio, init, em, er)
eng._encode()
for _ in range(steps):
    eng._step()
torch.cuda.synchronize()
print("pmc_step done", nw, steps)
