"""Dump LoFTR features (coarse, fine) of 8 seeded frames to an npz (A/B diagnostics):
    python tools/lf_feat_dump.py OUT.npz [--hw 480x640]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-level-indoor-slam_amd")]
from mlgate import synthetic  # noqa: E402
from mlgate.loftr import LoFTRGPU  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--hw", default="480x640")
a = ap.parse_args()
Hi, Wi = (int(x) for x in a.hw.split("x"))
seq = synthetic.make_sequence(8, 4, 0)
fr = torch.from_numpy(synthetic.frames_host(seq, np.arange(8), Hi, Wi)).to("cuda")
lf = LoFTRGPU(device=torch.device("cuda"))
c, f = lf.features(fr)
torch.cuda.synchronize()
np.savez(a.out, coarse=c.float().cpu().numpy(), fine=f.float().cpu().numpy())
print("saved", a.out, tuple(c.shape), tuple(f.shape))
