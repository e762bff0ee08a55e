"""LoFTR (configs[4]) timing on the GPU box: backbone per keyframe and matching per pair
on synthetic revisit pairs, HIP-event timed (python tools/loftr_bench.py [--hw 540x720]).
`digest` hashes counts, keypoints and confidences (bit identity of A/B arms); `kdigest`
counts and keypoints only (the same matches when an arm changes conf's last bits)."""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-level-indoor-slam_amd")]
from mlgate import synthetic  # noqa: E402
from mlgate.loftr import LoFTRGPU  # noqa: E402


def digest(n, k0, k1, cf):
    """hash of every pair's matches (counts, keypoints, confidences): bit-identity of A/B arms"""
    h = hashlib.sha256(n.cpu().numpy().tobytes())
    for p, c in enumerate(n.tolist()):
        for t in (k0[p, :c], k1[p, :c], cf[p, :c]):
            h.update(t.contiguous().cpu().numpy().tobytes())
    return h.hexdigest()[:16]


def kdigest(n, k0, k1):
    h = hashlib.sha256(n.cpu().numpy().tobytes())
    for p, c in enumerate(n.tolist()):
        for t in (k0[p, :c], k1[p, :c]):
            h.update(t.contiguous().cpu().numpy().tobytes())
    return h.hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--pairs", type=int, default=32)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--hw", default="480x640", help="frame H x W (540x720: the ISEC camera, network 536 x 720)")
    a = ap.parse_args()
    Hi, Wi = (int(x) for x in a.hw.split("x"))
    H, W = Hi // 8 * 8, Wi // 8 * 8
    dev = torch.device("cuda")
    seq = synthetic.make_sequence(a.frames, max(2, a.frames // 4), 0)
    fr = torch.from_numpy(synthetic.frames_host(seq, np.arange(a.frames), Hi, Wi)).to(dev)
    lf = LoFTRGPU(device=dev)
    po = seq.place_of
    pairs = [(i, j) for i in range(a.frames) for j in range(i + 1, a.frames) if po[i] == po[j]][:a.pairs]
    coarse, fine = lf.features(fr)
    n, *_ = lf.match_device(coarse, fine, H, W, [p for p, _ in pairs], [q for _, q in pairs])
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    for _ in range(a.iters):
        coarse, fine = lf.features(fr)
    e[1].record()
    for _ in range(a.iters):
        n, k0, k1, cf = lf.match_device(coarse, fine, H, W, [p for p, _ in pairs], [q for _, q in pairs])
    e[2].record()
    torch.cuda.synchronize()
    feat_ms = e[0].elapsed_time(e[1]) / a.iters
    match_ms = e[1].elapsed_time(e[2]) / a.iters
    gflop_feat = 2 * (240 * 320 * 49 * 128 + 240 * 320 * 9 * 128 * 128 * 4 + 120 * 160 * 9 * (128 * 196 + 3 * 196 * 196)
                      + 120 * 160 * 196 * 128 + 60 * 80 * 9 * (196 * 256 + 3 * 256 * 256) + 60 * 80 * 196 * 256
                      + 60 * 80 * 256 * 256 + 120 * 160 * (196 * 256 + 9 * 256 * 256 + 9 * 256 * 196)
                      + 240 * 320 * (128 * 196 + 9 * 196 * 196 + 9 * 196 * 128)) / 1e9
    print(json.dumps({"frames": a.frames, "pairs": len(pairs), "features_ms_per_frame": round(feat_ms / a.frames, 3),
                      "backbone_gflop_per_frame": round(gflop_feat, 1),
                      "backbone_tflops": round(gflop_feat * a.frames / feat_ms, 1),
                      "match_ms_per_pair": round(match_ms / len(pairs), 3),
                      "matches_mean": float(n.float().mean()), "digest": digest(n, k0, k1, cf),
                      "kdigest": kdigest(n, k0, k1), "frame": f"{Wi}x{Hi} (network {W}x{H})"}), flush=True)


if __name__ == "__main__":
    main()
