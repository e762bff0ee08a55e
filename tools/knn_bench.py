"""Time the all-keyframes kNN gate (mlg_knn_gate) at bench sizes: N keyframes x D, top-k,
time gap 10 s, threshold 0.5, floor gating -- the fused scan for k <= 32.  Prints the
per-call time and the algorithmic HBM bytes per call (each pass reads the normalised
descriptor matrix once per 64-row query block's column split, i.e. the database once
per row block from L2/HBM; algorithmic = raw descriptors read + normalised written +
re-read once = 3 N D 4 B)."""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-level-indoor-slam_amd")]
from mlgate import retrieval  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=5000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    rng = np.random.default_rng(0)
    X = torch.from_numpy(rng.standard_normal((a.n, a.d)).astype(np.float32)).to(dev)
    t = torch.from_numpy(np.arange(a.n) * 0.765).to(dev)
    fl = torch.from_numpy(rng.integers(1, 5, a.n).astype(np.int64)).to(dev)
    hf = torch.ones(a.n, dtype=torch.uint8, device=dev)
    retrieval.knn_gate(X, t, fl, hf, 10.0, 0.5, a.k, True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        retrieval.knn_gate(X, t, fl, hf, 10.0, 0.5, a.k, True)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    flops = 2.0 * a.n * a.n * a.d
    print(f"knn_gate N={a.n} D={a.d} k={a.k}: {ms:.3f} ms per call, {flops / ms / 1e9:.1f} TFLOP/s (exact-f32 MFMA), "
          f"{3 * a.n * a.d * 4 / ms / 1e6:.1f} GB/s algorithmic", flush=True)


if __name__ == "__main__":
    main()
