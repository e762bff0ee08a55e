"""Projected per-rank step of the frame-sharded gate at W ranks, measured on ONE GPU
(VERDICT r04 "next 7": multi-GPU readiness without an 8-GPU node).

bench.py's workload (5000 keyframes, 600 places, k = 20).  A world-1 DeviceGate runs one
full step first (it fills the SuperPoint feature table of every keyframe and yields the
global verification pair list).  Then each rank r's share of a W-rank step is timed on
this GPU, stage by stage, exactly as DeviceGate(world=W, rank=r) would run it:
  * ViT + GeM on its keyframes [r N / W, (r + 1) N / W) (VitB14, split forward, batch 246);
  * the fused kNN + floor gate of its query rows against all N descriptors;
  * SuperPoint on its keyframes (batch 64);
  * LightGlue + RANSAC + decisions on its slice of the pair list: balanced_pairs with
    group_reverse (the unordered pairs split evenly in (min, max) order, as
    mlgate.distributed does), one LightGlue call for the slice (DeviceGate._verify_lightglue
    over the features of every keyframe, which is what FeatureExchange hands the rank).
The exchange steps are not run (one GPU); their bytes are computed from the slice and
priced at an assumed xGMI rate (--xgmi-gbs, per rank, receive side):
  * the descriptor all-gather: (W - 1) / W x N x 768 x 4 B per rank;
  * FeatureExchange: the SuperPoint features (2048 x 2 + 2048 x 256 float32 + a count) of
    every keyframe the slice touches that the rank does not own.
The step of the sharded run is the slowest rank's; efficiency = T(1) / (W x max_r T(r)).
This is a projection: no collective ran and no second GPU was involved.

    python tools/rank_projection.py [--world 8] [--reps 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-level-indoor-slam_amd")]

import bench  # noqa: E402
from mlgate import distributed as mdist  # noqa: E402
from mlgate import retrieval, synthetic  # noqa: E402
from mlgate.pipeline import DeviceGate  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402

FEATURE_BYTES = 2048 * 2 * 4 + 2048 * 256 * 4 + 4  # kp f32 + desc f32 + count, per keyframe


def log(**kw):
    print(json.dumps(kw), flush=True)


def timed(fn, reps):
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    return best


def rank_slice(pa, pb, world, rank):
    """balanced_pairs(group_reverse=True) on host arrays: the rank's ordered pairs."""
    lo_, hi_ = np.minimum(pa, pb).astype(np.int64), np.maximum(pa, pb).astype(np.int64)
    ukey, inv = np.unique(lo_ * (int(hi_.max()) + 1) + hi_, return_inverse=True)
    nu = len(ukey)
    u0, u1 = rank * nu // world, (rank + 1) * nu // world
    sel = np.flatnonzero((inv >= u0) & (inv < u1))
    return pa[sel], pb[sel], u1 - u0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--keyframes", type=int, default=5000)
    ap.add_argument("--places", type=int, default=600)
    ap.add_argument("--xgmi-gbs", type=float, default=300.0,
                    help="assumed receive rate per rank for the exchanges (GB/s; 7 xGMI links)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N, W = a.keyframes, a.world
    seq, labels = bench.sequence(N, a.places)
    frames = synthetic.frames_device(seq, np.arange(N), dev)
    gate = DeviceGate(frames, seq.t, labels, 1, 0, dev, k=20, verify=True, K=bench.ISEC_K, vit_batch=246,
                      sp_batch=64, lg_chunk=5120, vit_state_dict=synthetic_state_dict(0))
    gate.step()  # warm-up, fills every keyframe's SuperPoint features
    t1 = timed(gate.step, a.reps)
    pa, pb = gate.last_pairs
    log(phase="world1", step_s=round(t1, 3), pairs=len(pa))
    eng = gate.eng
    rows = []
    for r in range(W):
        lo, hi = mdist.shard(N, W, r)
        n_loc = hi - lo
        desc = torch.empty(n_loc, 768, device=dev)
        local = torch.empty(n_loc, eng.n_local, 768, device=dev)
        t_vit = timed(lambda: eng.forward_into(frames[lo:hi], desc, local), a.reps)
        totals = torch.zeros(2, dtype=torch.int64, device=dev)
        t_knn = timed(lambda: retrieval.knn_gate(gate.gather.out, gate.t_all, gate.f_all, gate.hf_all, gate.gap,
                                                 gate.thr, gate.k, True, q0=lo, Q=n_loc, totals=totals), a.reps)

        def sp():
            for b0 in range(lo, hi, 64):
                b1 = min(hi, b0 + 64)
                gate.sp.extract_device(frames[b0:b1])
        t_sp = timed(sp, a.reps)
        spa, spb, nu = rank_slice(pa, pb, W, r)
        out = {}
        t_ver = timed(lambda: gate._verify_lightglue(spa, spb, True, out), a.reps)
        need = np.unique(np.concatenate([spa, spb]))
        remote = int(((need < lo) | (need >= hi)).sum())
        x_bytes = (W - 1) / W * N * 768 * 4 + remote * FEATURE_BYTES
        t_x = x_bytes / (a.xgmi_gbs * 1e9)
        row = {"rank": r, "keyframes": n_loc, "ordered_pairs": len(spa), "unordered_pairs": int(nu),
               "vit_s": round(t_vit, 4), "knn_s": round(t_knn, 4), "superpoint_s": round(t_sp, 4),
               "verify_s": round(t_ver, 4), "remote_keyframes": remote, "exchange_gb": round(x_bytes / 1e9, 3),
               "exchange_s_at_assumed_rate": round(t_x, 4),
               "step_s": round(t_vit + t_knn + t_sp + t_ver + t_x, 4)}
        log(**row)
        rows.append(row)
    tmax = max(r_["step_s"] for r_ in rows)
    rep = {"world": W, "t1_s": round(t1, 3), "t1_over_w_s": round(t1 / W, 4), "projected_step_s": tmax,
           "projected_kf_per_s": round(N / tmax, 1), "projected_efficiency": round(t1 / (W * tmax), 3),
           "xgmi_gbs_assumed": a.xgmi_gbs,
           "compute_only_efficiency": round(t1 / (W * max(r_["step_s"] - r_["exchange_s_at_assumed_rate"]
                                                           for r_ in rows)), 3)}
    log(**rep)


if __name__ == "__main__":
    main()
