"""Dump GPU restore output for the test cases (gpurun_out/restore_dbg.npz)."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_restore import CASES, _frames, _faces, align_matrix
from latentsync_amd import restore as RS
n = len(CASES)
frames, faces = _frames(n), _faces(n)
mats = [align_matrix(*c) for c in CASES]
fr = torch.from_numpy(frames).cuda()
RS.AlignRestore("cuda").restore_frames(fr, torch.from_numpy(faces).cuda(), mats)
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/restore_dbg.npz", out=fr.cpu().numpy())
print("saved")
