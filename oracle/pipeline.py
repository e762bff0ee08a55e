"""Oracle for the full semantic gate (test infrastructure only).

The CPU chain SURVEY.md §3.5 defines, built from the restatements in this package:
IMU floor labels (oracle.floors: floor_detector.py:63-156) -> CricaVPR descriptors
(oracle.vit, fp32: place_recognition.py:613-643, 781-803) -> find_loop_closures
(oracle.retrieval: :851-911) -> verify_with_semantics on every match with is_valid
(geometric_verification.py:688-734: the cross-floor skip, SuperPoint + LightGlue in
fp32 (oracle.superpoint / oracle.lightglue, emulate_bf16=False), OpenCV's RANSAC loop
(oracle.geometry.cv_ransac) and the decision rule :606-620) -> the floor gate on the
geometrically valid pairs (oracle.gate: loop_closure_gate.py:60-126) -> the four-term
false-loop-closure rejection count.
"""
import numpy as np
import torch

from . import floors as ofl
from . import gate as ogate
from . import geometry as ogeo
from . import lightglue as olg
from . import retrieval as oret
from . import superpoint as osp
from . import vit as ovit


def floor_codes(labels):
    """Reference equality semantics of `query_floor == match_floor` as integer codes
    (labels here are ints: identity)."""
    return np.asarray(labels, np.int64), np.ones(len(labels), np.uint8)


def descriptors(frames, vit_sd):
    sd = {k: torch.as_tensor(np.asarray(v)) for k, v in vit_sd.items()}
    return np.stack([ovit.extract_descriptor(f, sd) for f in frames]).astype(np.float32)


def verify_pair(img_a, img_b, sp_sd, lg, K, max_kp=2048, min_inliers=20, min_inlier_ratio=0.25, thr=3.0,
                feats=None):
    """GeometricVerifier.verify (geometric_verification.py:564-634) in fp32 with the
    oracle matcher; returns dict(num_matches, num_inliers, inlier_ratio, is_valid,
    matches)."""
    fa, fb = feats if feats is not None else osp.superpoint(sp_sd, [img_a, img_b], max_kp=max_kp,
                                                            emulate_bf16=False)
    r = lg.match(fa["keypoints"], fa["descriptors"], fb["keypoints"], fb["descriptors"])
    mm = r["matches"].numpy()
    k1 = fa["keypoints"].numpy()[mm[:, 0]].astype(np.float32)
    k2 = fb["keypoints"].numpy()[mm[:, 1]].astype(np.float32)
    n = len(k1)
    if n < 5:
        return {"num_matches": 0, "num_inliers": 0, "inlier_ratio": 0.0, "is_valid": False, "matches": mm,
                "stop": r["stop"]}
    _, mask, n_in = ogeo.cv_ransac(k1, k2, K, thr)
    ratio = float(np.sum(mask) / n)
    return {"num_matches": n, "num_inliers": int(n_in), "inlier_ratio": ratio,
            "is_valid": bool(n_in >= min_inliers and ratio >= min_inlier_ratio), "matches": mm, "stop": r["stop"]}


def gate_chain(labels, X, t, K, verify_fn, min_gap=10.0, thr=0.5, k=10, retrieval_gating=True,
               verifier_gating=True, strict=True):
    """Stages 3-5 given labels, descriptors and a per-pair verifier (q, m) -> dict."""
    codes, has = floor_codes(labels)
    q, m, sim, valid = oret.find_loop_closures(X, t, codes, has, min_gap, thr, k, retrieval_gating)
    valid = np.asarray(valid, bool)
    vq, vm = q[valid], m[valid]
    skip = np.array([verifier_gating and labels[a] != labels[b] for a, b in zip(vq, vm)], bool)
    res = [None if s else verify_fn(int(a), int(b)) for a, b, s in zip(vq, vm, skip)]
    ok = np.array([r is not None and r["is_valid"] for r in res], bool)
    gvalid, _, _ = ogate.gate_decisions(labels, vq[ok], vm[ok], strict) if ok.any() else (np.zeros(0, bool), 0, 0)
    counts = {"retrieval_floor_rejected": int((~valid).sum()), "skipped_floor_mismatch": int(skip.sum()),
              "verifier_invalid": int(sum(1 for r in res if r is not None and not r["is_valid"])),
              "gate_rejected_cross_floor": int((~np.asarray(gvalid, bool)).sum())}
    counts["total"] = sum(counts.values())
    return {"q": q, "m": m, "sim": sim, "valid": valid, "skip": skip, "results": res, "geo_valid": ok,
            "gate_valid": np.asarray(gvalid, bool), "counts": counts}


def floor_labels(timestamps, imu, start_floor=5):
    t, ax, ay, az = imu[:4]
    return ofl.assign_labels(timestamps, ofl.detect_events(t, ax, ay, az), start_floor)


def make_matcher(lg_sd):
    return olg.Oracle(lg_sd, emulate_bf16=False)
