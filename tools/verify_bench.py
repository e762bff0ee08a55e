"""Throughput of the verification stage (GPU box tool): SuperPoint on a batch of
synthetic keyframes, LightGlue on pairs of them, batched RANSAC + recoverPose.

    python tools/verify_bench.py [--frames 64] [--pairs 64] [--iters 3]

Prints one JSON line per stage with HIP-event milliseconds.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
sys.path.insert(0, ROOT)

from mlgate import synthetic  # noqa: E402
from mlgate import geometry  # noqa: E402
from mlgate.lightglue import LightGlueGPU  # noqa: E402
from mlgate.superpoint import SuperPointGPU  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(iters):
        out = fn()
    e1.record()
    torch.cuda.synchronize()
    return out, e0.elapsed_time(e1) / iters, (time.perf_counter() - t0) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    F = args.frames
    seq = synthetic.make_sequence(F, max(F // 2, 1), 0)  # each place seen about twice
    frames = synthetic.frames_device(seq, np.arange(F), dev)
    sp = SuperPointGPU(device=dev)
    (kp, sc, ds, _, cnt), ms, wall = timed(lambda: sp.extract_device(frames), args.iters)
    counts = cnt.cpu().numpy()
    import hashlib
    h = hashlib.sha1()
    for t in (kp, sc, ds, cnt):
        h.update(t.float().cpu().numpy().tobytes())
    print(json.dumps({"stage": "superpoint", "frames": F, "ms": round(ms, 3), "wall_ms": round(wall, 3),
                      "sha1": h.hexdigest()[:16],
                      "frames_per_s": round(F / ms * 1e3, 1), "mean_keypoints": float(counts.mean()),
                      "gflop_per_frame": 52.1}), flush=True)
    rng = np.random.default_rng(0)
    pa = rng.integers(0, F, args.pairs)
    pb = (pa + rng.integers(1, F, args.pairs)) % F
    lg = LightGlueGPU(device=dev)
    (m, s, n, stop), ms, wall = timed(lambda: lg.match_device(kp, ds, counts, pa, pb), args.iters)
    nm = n.cpu().numpy()
    print(json.dumps({"stage": "lightglue", "pairs": args.pairs, "ms": round(ms, 3), "wall_ms": round(wall, 3),
                      "pairs_per_s": round(args.pairs / wall * 1e3, 1), "mean_matches": float(nm.mean()),
                      "mean_layers": float(np.mean(stop))}), flush=True)
    kpn, mn = kp.cpu().numpy(), m.cpu().numpy()
    k1 = [kpn[a][mn[p, :nm[p], 0]] for p, a in enumerate(pa)]
    k2 = [kpn[b][mn[p, :nm[p], 1]] for p, b in enumerate(pb)]
    K = np.array([[893.63, 0, 376.95], [0, 893.97, 266.57], [0, 0, 1.0]])
    res, ms, wall = timed(lambda: geometry.epipolar_ransac(k1, k2, K, 3.0, device=str(dev)), args.iters)
    print(json.dumps({"stage": "ransac", "pairs": args.pairs, "ms": round(ms, 3), "wall_ms": round(wall, 3),
                      "pairs_per_s": round(args.pairs / wall * 1e3, 1),
                      "mean_inliers": float(np.mean([r.inliers for r in res]))}), flush=True)


if __name__ == "__main__":
    main()
