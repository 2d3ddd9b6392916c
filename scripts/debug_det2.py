"""Bitwise run-to-run determinism of the full UNet forward (8 windows) and of the tiled GEMMs."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from latentsync_amd.config import STAGE2_MODEL
from latentsync_amd.unet import UNet3DConditionModel
unet = UNet3DConditionModel(**STAGE2_MODEL).init_weights(41).to("cuda").eval()
g = torch.Generator().manual_seed(0)
x = torch.randn((8, 13, 16, 32, 32), generator=g).cuda()
a = torch.randn((128, 50, 384), generator=g).cuda()
outs = []
with torch.no_grad():
    for _ in range(4):
        outs.append(unet(x, 951, encoder_hidden_states=a).sample.clone())
print("unet fwd differing elements vs run0:", [int((o != outs[0]).sum()) for o in outs],
      "max abs diff:", [float((o - outs[0]).abs().max()) for o in outs])
