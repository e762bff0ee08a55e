"""Time the batched epipolar RANSAC (mlg_ransac_epipolar) on bench-like pairs: P pairs of
S matches with a given inlier fraction (low fractions keep OpenCV's loop at its full
1000 iterations, as non-revisit pairs do in bench.py)."""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-level-indoor-slam_amd")]
from mlgate import geometry  # noqa: E402
from oracle import geometry as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--matches", type=int, default=1700)
    ap.add_argument("--inliers", type=float, default=0.2)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    n_in = int(a.matches * a.inliers)
    k1s, k2s = [], []
    for _ in range(8):
        k1, k2, *_ = G.synthetic_pair(rng, n_in, a.matches - n_in, 0.5)
        k1s.append(k1)
        k2s.append(k2)
    k1 = np.concatenate([k1s[i % 8] for i in range(a.pairs)])
    k2 = np.concatenate([k2s[i % 8] for i in range(a.pairs)])
    offs = np.arange(a.pairs + 1, dtype=np.int32) * a.matches
    dev = torch.device("cuda")
    K = torch.from_numpy(G.ISEC_K.reshape(9).copy()).to(dev)
    args = (torch.from_numpy(k1).to(dev), torch.from_numpy(k2).to(dev), torch.from_numpy(offs).to(dev), K, 0, 3.0)
    geometry.epipolar_ransac_device(*args)
    torch.cuda.synchronize()
    best = None
    for _ in range(a.reps):
        t0 = time.perf_counter()
        out = geometry.epipolar_ransac_device(*args)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    h = hashlib.sha1()
    for t in out:
        if isinstance(t, torch.Tensor):
            h.update(t.cpu().numpy().tobytes())
    print(json.dumps({"pairs": a.pairs, "matches": a.matches, "inliers": a.inliers, "ms": round(best * 1e3, 2),
                      "mean_inliers": round(out[2].float().mean().item(), 3), "digest": h.hexdigest()[:16]}),
          flush=True)


if __name__ == "__main__":
    main()
