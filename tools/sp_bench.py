"""SuperPoint stage microbenchmark (GPU box tool).

    python tools/sp_bench.py [--frames 64] [--iters 5]

bench.py's synthetic 640x480 keyframes through SuperPointGPU.extract_device (conv stack,
scores, NMS, top-k selection, descriptors) in one batch, timed with HIP events; prints the
time per keyframe and a digest of every output (keypoints, scores, descriptors, counts)
for bit-identity checks across builds.
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
sys.path.insert(0, ROOT)

from mlgate import synthetic  # noqa: E402
from mlgate.superpoint import SuperPointGPU  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    seq = synthetic.make_sequence(args.frames, max(2, args.frames // 4), 0)
    frames = synthetic.frames_device(seq, np.arange(args.frames), dev)
    sp = SuperPointGPU(device=dev, max_num_keypoints=2048)
    out = sp.extract_device(frames)  # warm-up
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        out = sp.extract_device(frames)
    e1.record()
    torch.cuda.synchronize()
    kp, sc, ds, _, cnt = out
    h = hashlib.sha1()
    for t in (kp, sc, ds, cnt):
        h.update(t.cpu().numpy().tobytes())
    print(json.dumps({"frames": args.frames, "ms_per_keyframe": round(e0.elapsed_time(e1) / args.iters / args.frames, 4),
                      "mean_keypoints": float(cnt.float().mean()), "digest": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
