"""SuperGlue stage microbenchmark (GPU box tool).

    python tools/sg_bench.py [--pairs 256] [--frames 64] [--iters 3]

SuperPoint features (magicleap settings: threshold 0.005, 2048 keypoints) of bench.py's
synthetic keyframes, then SuperGlue (18 GNN layers + 20 Sinkhorn iterations) on `pairs`
random pairs in one call, timed with HIP events.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
sys.path.insert(0, ROOT)

from mlgate import synthetic  # noqa: E402
from mlgate.superglue import SuperGlueGPU  # noqa: E402
from mlgate.superpoint import SuperPointGPU  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    seq = synthetic.make_sequence(args.frames, max(2, args.frames // 4), 0)
    frames = synthetic.frames_device(seq, np.arange(args.frames), dev)
    kp, sc, ds, _, cnt = SuperPointGPU(device=dev, max_num_keypoints=2048,
                                       detection_threshold=0.005).extract_device(frames)
    counts = cnt.cpu().numpy()
    rng = np.random.default_rng(0)
    pa = rng.integers(0, args.frames, args.pairs).astype(np.int32)
    pb = ((pa + rng.integers(1, args.frames, args.pairs)) % args.frames).astype(np.int32)
    sg = SuperGlueGPU(device=dev)
    W, H = int(frames.shape[2]), int(frames.shape[1])
    m, s, n = sg.match_device(kp, sc, ds, counts, pa, pb, W, H)  # warm-up
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        m, s, n = sg.match_device(kp, sc, ds, counts, pa, pb, W, H)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    print(json.dumps({"pairs": args.pairs, "mean_keypoints": float(counts.mean()), "ms_per_call": round(ms, 2),
                      "ms_per_pair": round(ms / args.pairs, 4), "matches_mean": float(n.float().mean())}))


if __name__ == "__main__":
    main()
