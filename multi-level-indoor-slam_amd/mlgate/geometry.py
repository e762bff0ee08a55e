"""Batched epipolar RANSAC + relative pose on the GPU (``mlg_ransac_epipolar`` /
``mlg_recover_pose``, include/mlgate.h).

Replaces the OpenCV calls of BaseFeatureMatcher.verify_geometric_consistency and
estimate_relative_pose (scripts/semantic_gating/geometric_verification.py:104-188)
for any number of candidate pairs in one launch sequence.
"""
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native

DEFAULT_HYPOTHESES = 1000  # OpenCV's maxIters for findEssentialMat / findFundamentalMat


@dataclass
class RansacResult:
    mask: np.ndarray             # bool [S]
    model: Optional[np.ndarray]  # 3x3 E (K given) or F; None when no model
    inliers: int
    pose: Optional[np.ndarray]   # 4x4 [R|t] (E path, >= 5 inliers) else None
    status: int                  # 0 ok, 1 no model, 2 model but < 5 inliers


def _flat(pairs_k1, pairs_k2):
    sizes = [len(a) for a in pairs_k1]
    if [len(b) for b in pairs_k2] != sizes:
        raise ValueError("kpts1 / kpts2 lengths differ")
    offs = np.zeros(len(sizes) + 1, np.int32)
    np.cumsum(sizes, out=offs[1:])
    k1 = np.concatenate([np.asarray(a, np.float32).reshape(-1, 2) for a in pairs_k1]) if sizes else np.zeros((0, 2),
                                                                                                          np.float32)
    k2 = np.concatenate([np.asarray(b, np.float32).reshape(-1, 2) for b in pairs_k2]) if sizes else np.zeros((0, 2),
                                                                                                          np.float32)
    return k1, k2, offs


def _k_tensor(K, P, dev):
    if K is None:
        return None, 0
    K = np.asarray(K, np.float64)
    if K.shape == (3, 3):
        return torch.from_numpy(K.reshape(9).copy()).to(dev), 0
    return torch.from_numpy(K.reshape(P, 9).copy()).to(dev), 9


def epipolar_ransac_device(k1, k2, offs, K=None, k_stride=0, threshold=3.0, hypotheses=DEFAULT_HYPOTHESES, seed=0,
                           with_pose=True):
    """Device entry: k1, k2 float32 [S, 2], offs int32 [P + 1], K float64 (9 or P*9) or None.

    Returns device tensors (model [P, 9] f64, mask [S] u8, inliers [P] i32, pose [P, 16] f64 or None,
    status [P] i32).
    """
    model, mask, inl, pose, status = _native.ops().ransac_epipolar(
        k1.contiguous(), k2.contiguous(), offs.contiguous(), K, int(k_stride), float(threshold), int(hypotheses),
        int(seed) & ((1 << 63) - 1), bool(with_pose))
    return model, mask, inl, (pose if pose.numel() else None), status


def epipolar_ransac(pairs_k1: Sequence[np.ndarray], pairs_k2: Sequence[np.ndarray], K=None, threshold: float = 3.0,
                    hypotheses: int = DEFAULT_HYPOTHESES, seed: int = 0, device: str = "cuda",
                    with_pose: bool = True) -> List[RansacResult]:
    """Host entry: lists of per-pair matched keypoints (pixels) -> one RansacResult per pair.

    K: None (fundamental matrix), a 3x3 intrinsic matrix shared by all pairs, or [P, 3, 3].
    """
    dev = _native.require_device(device)
    k1, k2, offs = _flat(pairs_k1, pairs_k2)
    P = len(offs) - 1
    if P == 0:
        return []
    Kt, ks = _k_tensor(K, P, dev)
    model, mask, inl, pose, status = epipolar_ransac_device(
        torch.from_numpy(k1).to(dev), torch.from_numpy(k2).to(dev), torch.from_numpy(offs).to(dev), Kt, ks,
        threshold, hypotheses, seed, with_pose)
    model, mask, inl, status = model.cpu().numpy(), mask.cpu().numpy().astype(bool), inl.cpu().numpy(), \
        status.cpu().numpy()
    pose = pose.cpu().numpy() if pose is not None else None
    out = []
    for p in range(P):
        st = int(status[p])
        out.append(RansacResult(mask=mask[offs[p]:offs[p + 1]].copy(),
                                model=None if st == 1 else model[p].reshape(3, 3).copy(), inliers=int(inl[p]),
                                pose=pose[p].reshape(4, 4).copy() if (pose is not None and st == 0) else None,
                                status=st))
    return out


def recover_pose(kpts1, kpts2, K, inlier_mask, E, device: str = "cuda") -> Optional[np.ndarray]:
    """cv2.recoverPose(E, kpts1[mask], kpts2[mask], K) as a 4x4 [R|t; 0 0 0 1]; None below 5 inliers."""
    mask = np.asarray(inlier_mask, bool)
    if E is None or mask.sum() < 5:
        return None
    dev = _native.require_device(device)
    k1, k2, offs = _flat([kpts1], [kpts2])
    k1, k2, offs = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (k1, k2, offs))
    K = torch.from_numpy(np.asarray(K, np.float64).reshape(9).copy()).to(dev)
    E = torch.from_numpy(np.asarray(E, np.float64).reshape(9).copy()).to(dev)
    m = torch.from_numpy(mask.astype(np.uint8)).to(dev)
    return _native.ops().recover_pose(k1, k2, offs, K, 0, E, m).cpu().numpy().reshape(4, 4)
