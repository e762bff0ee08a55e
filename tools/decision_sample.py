"""Bench-scale verifier decisions for the fp32 cross-check (GPU box tool; VERDICT r02
item 3).

    python tools/decision_sample.py [--keyframes 5000] [--sample 600] [--out gpurun_out/decision_sample.npz]

Runs bench.py's full gate once (DeviceGate, N keyframes, k = 20, record=True) on
keyframes generated on the HOST (mlgate.synthetic.frames_host: numpy noise, so the CPU
can regenerate any keyframe bit for bit), and saves, for a seeded uniform sample of the
step's verified ordered pairs (no margin filter), the GPU's per-pair LightGlue match
count, RANSAC inlier count and decision.  tools/decision_check_cpu.py then recomputes
the same pairs with the fp32 chain (oracle.pipeline.verify_pair: SuperPoint + LightGlue
fp32, OpenCV's RANSAC loop restated) and reports the decision flip rate."""
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

import bench  # noqa: E402
from mlgate import synthetic  # noqa: E402
from mlgate.pipeline import DeviceGate  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402

SAMPLE_SEED = 2026


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keyframes", type=int, default=5000)
    ap.add_argument("--places", type=int, default=600)
    ap.add_argument("--sample", type=int, default=600)
    ap.add_argument("--out", default="gpurun_out/decision_sample.npz")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    t0 = time.time()
    seq, labels = bench.sequence(a.keyframes, a.places)
    frames = torch.empty(a.keyframes, synthetic.H, synthetic.W, 3, dtype=torch.uint8, device=dev)
    for b0 in range(0, a.keyframes, 250):
        idx = np.arange(b0, min(a.keyframes, b0 + 250))
        frames[b0:b0 + len(idx)].copy_(torch.from_numpy(synthetic.frames_host(seq, idx)))
        print(json.dumps({"frames": int(idx[-1]) + 1, "s": round(time.time() - t0, 1)}), flush=True)
    gate = DeviceGate(frames, seq.t, labels, 1, 0, dev, k=20, verify=True, K=bench.ISEC_K, vit_batch=123, sp_batch=64,
                      lg_chunk=2048, vit_state_dict=synthetic_state_dict(0), record=True)
    counts = gate.step()
    r = gate.last_pair_results
    P = len(r["a"])
    rng = np.random.default_rng(SAMPLE_SEED)
    pick = np.sort(rng.choice(P, size=min(a.sample, P), replace=False))
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.savez_compressed(a.out, keyframes=a.keyframes, places=a.places, seq_seed=0, sample_seed=SAMPLE_SEED,
                        a=r["a"][pick], b=r["b"][pick], matches=r["matches"][pick], inliers=r["inliers"][pick],
                        is_valid=r["is_valid"][pick], pairs_total=P, valid_total=int(r["is_valid"].sum()),
                        counts=json.dumps(counts))
    print(json.dumps({"pairs_verified": P, "valid": int(r["is_valid"].sum()), "sample": int(len(pick)),
                      "sample_valid": int(r["is_valid"][pick].sum()), "counts": counts,
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
