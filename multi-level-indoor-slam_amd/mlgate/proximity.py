"""Trajectory-proximity loop-closure candidates with the floor gate fused in.

Drop-in for the candidate generator and gate of the SLAM integrations
(scripts/semantic_gating/orb_slam3_integration.py:167-281 and
lego_loam_integration.py:121-204: ``detect_loop_closure_candidates`` +
``apply_floor_gating`` + ``LoopClosureAnalysis``), computed by ``mlg_proximity_count``
/ ``mlg_proximity_emit`` (include/mlgate.h) instead of a KD-tree and Python loops.

Candidates are all (i, j) with i < j, j - i >= min_time_gap and
||p_i - p_j|| <= distance_threshold.  They come back in (i, j) order; the
reference's order within a row is the KD-tree's emission order, which carries no
meaning (its consumers only count them).  Counts, sets and verdicts are identical.
"""
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import _native
from .gate import SemanticLoopClosureGate


@dataclass
class LoopClosureAnalysis:
    """Results of apply_floor_gating (orb_slam3_integration.py:34-41).

    ``cross_floor_pairs`` holds rows (idx1, idx2, floor1, floor2); here it is an int64
    array [C, 4] rather than a list of tuples (len / slicing / unpacking behave alike).
    """
    total_candidates: int = 0
    same_floor_candidates: int = 0
    cross_floor_candidates: int = 0
    true_positive_rate: float = 0.0
    false_positive_rate: float = 0.0
    cross_floor_pairs: List[Tuple[int, int, int, int]] = field(default_factory=list)


class ProximityCandidates:
    """Candidate set on the host: pairs int64 [P, 2], dist float64 [P], valid bool [P]."""

    def __init__(self, pairs, dist, valid, accepted, strict_mode=True, gated=True):
        self.pairs, self.dist, self.valid, self.accepted = pairs, dist, valid, int(accepted)
        self.strict_mode, self.gated = bool(strict_mode), bool(gated)

    def __len__(self):
        return len(self.pairs)

    def to_list(self) -> List[Tuple[int, int, float]]:
        """The reference's return type: [(query_idx, match_idx, distance), ...]."""
        return [(int(i), int(j), float(d)) for (i, j), d in zip(self.pairs, self.dist)]


def _as_device(x, dtype, dev):
    t = torch.as_tensor(np.ascontiguousarray(x)) if not torch.is_tensor(x) else x
    return t.to(device=dev, dtype=dtype).contiguous()


def proximity_candidates_device(pos, floor=None, distance_threshold=2.0, min_time_gap=100, strict_mode=True,
                                row0=0, nrows=None):
    """Device entry: pos float64 [N, 3] and floor int64 [N] (or None) on the HIP device.

    Returns device tensors (pairs int32 [P, 2], dist float64 [P], valid uint8 [P]) and the
    host ints (candidates, accepted) for query rows [row0, row0 + nrows).
    """
    N = int(pos.shape[0])
    nrows = N - row0 if nrows is None else int(nrows)
    if N > 65536 or not 0 <= row0 <= N or nrows < 0 or row0 + nrows > N:
        raise ValueError(f"proximity search supports up to 65536 poses and a row range inside [0, N) "
                         f"(N={N}, row0={row0}, nrows={nrows})")
    pairs, dist, valid, totals = _native.ops().proximity(pos.contiguous(), floor, int(row0), nrows,
                                                         float(distance_threshold), int(min_time_gap),
                                                         bool(strict_mode))
    total, accepted = (int(v) for v in totals.cpu())
    return pairs[:total], dist[:total], valid[:total], total, accepted


def detect_loop_closure_candidates(positions, distance_threshold: float = 2.0, min_time_gap: int = 100,
                                   floor_labels: Optional[np.ndarray] = None, strict_mode: bool = True,
                                   device: str = "cuda") -> ProximityCandidates:
    """positions: [N, 3] metres (TUM columns 1..3).  Host arrays in, host arrays out."""
    if min_time_gap < 1:
        raise ValueError("min_time_gap must be >= 1 (the reference keeps only i < j)")
    dev = _native.require_device(device)
    pos = _as_device(np.asarray(positions, dtype=np.float64).reshape(-1, 3), torch.float64, dev)
    fl = None if floor_labels is None else _as_device(np.asarray(floor_labels, dtype=np.int64), torch.int64, dev)
    pairs, dist, valid, total, accepted = proximity_candidates_device(pos, fl, distance_threshold, min_time_gap,
                                                                      strict_mode)
    return ProximityCandidates(pairs.cpu().numpy().astype(np.int64), dist.cpu().numpy(),
                               valid.cpu().numpy().astype(bool), accepted, strict_mode, fl is not None)


def apply_floor_gating(candidates: ProximityCandidates, floor_labels: np.ndarray,
                       strict_mode: bool = True) -> Tuple[LoopClosureAnalysis, SemanticLoopClosureGate]:
    """The analysis and the gate (with its stats) of apply_floor_gating.

    The verdicts computed in the kernel are used when ``candidates`` were generated
    with floor labels and the same strict_mode (pass the same labels); otherwise the
    gate's vectorised decide() recomputes them.
    """
    f = np.asarray(floor_labels)
    gate = SemanticLoopClosureGate(f, strict_mode=strict_mode)
    pairs = candidates.pairs
    fq, fm = f[pairs[:, 0]], f[pairs[:, 1]]
    cross = fq != fm  # the analysis counts strict inequality whatever the gate mode (:241-250)
    a = LoopClosureAnalysis(total_candidates=len(pairs), same_floor_candidates=int(len(pairs) - cross.sum()),
                            cross_floor_candidates=int(cross.sum()))
    a.cross_floor_pairs = np.stack([pairs[cross, 0], pairs[cross, 1], fq[cross], fm[cross]], axis=1).astype(np.int64)
    n = len(pairs)
    if candidates.gated and candidates.strict_mode == bool(strict_mode):
        acc = candidates.accepted
    else:
        acc = int(gate.decide(pairs[:, 0], pairs[:, 1]).sum()) if n else 0
    gate.stats.update(total_candidates=n, accepted=acc, rejected_cross_floor=n - acc)
    return a, gate


class TrajectoryLoopClosureGate:
    """Positions + floor labels in, gated proximity candidates out: the compute core of
    ORBSlam3SemanticIntegration / LegoLoamSemanticIntegration without their file
    loading and plotting (orb_slam3_integration.py:167-281)."""

    def __init__(self, positions, floor_labels, device: str = "cuda"):
        self.positions = np.asarray(positions, dtype=np.float64).reshape(-1, 3)
        self.floor_labels = np.asarray(floor_labels)
        self.device = device
        self.loop_gate = None

    def detect_loop_closure_candidates(self, distance_threshold: float = 2.0, min_time_gap: int = 100,
                                       strict_mode: bool = True) -> ProximityCandidates:
        return detect_loop_closure_candidates(self.positions, distance_threshold, min_time_gap, self.floor_labels,
                                              strict_mode, self.device)

    def apply_floor_gating(self, candidates: ProximityCandidates, strict_mode: bool = True) -> LoopClosureAnalysis:
        analysis, self.loop_gate = apply_floor_gating(candidates, self.floor_labels, strict_mode)
        return analysis
