"""Floor-consistency loop-closure gate: drop-in mirror of
scripts/semantic_gating/loop_closure_gate.py (SemanticLoopClosureGate,
LoopClosureCandidate, ContextualPriorFactor, integrate_with_orbslam3).

On the hot path the gate decision is fused into the kNN kernel's epilogue
(knn.hip: k_topk_gate).  This class is the standalone host-side API for candidate
lists produced elsewhere; decisions are computed for the whole batch at once and the
per-candidate objects are built afterwards, in input order, with the reference's
stats keys, rejection reasons and counters.
"""
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np


@dataclass
class LoopClosureCandidate:
    """One gated (query, match) candidate and its verdict."""
    query_idx: int
    match_idx: int
    similarity_score: float
    query_floor: int
    match_floor: int
    is_valid: bool = True
    rejection_reason: str = ""


class SemanticLoopClosureGate:
    """Strict mode rejects any floor difference; non-strict rejects differences > 1."""

    def __init__(self, floor_labels: np.ndarray, strict_mode: bool = True):
        self.floor_labels = floor_labels
        self.strict_mode = strict_mode
        self.stats = {'total_candidates': 0, 'accepted': 0, 'rejected_cross_floor': 0, 'rejected_other': 0}

    def _reason(self, qf, mf):
        return f"Cross-floor: {qf} vs {mf}" if self.strict_mode else f"Floor diff > 1: {qf} vs {mf}"

    def _limit(self):
        return 0 if self.strict_mode else 1

    def gate_candidate(self, query_idx: int, match_idx: int, similarity_score: float = 0.0) -> LoopClosureCandidate:
        qf, mf = self.floor_labels[query_idx], self.floor_labels[match_idx]
        c = LoopClosureCandidate(query_idx=query_idx, match_idx=match_idx, similarity_score=similarity_score,
                                 query_floor=qf, match_floor=mf)
        self.stats['total_candidates'] += 1
        if abs(qf - mf) > self._limit():
            c.is_valid = False
            c.rejection_reason = self._reason(qf, mf)
            self.stats['rejected_cross_floor'] += 1
        else:
            self.stats['accepted'] += 1
        return c

    def decide(self, query_idx, match_idx) -> np.ndarray:
        """Vectorised verdicts (True = accept) for index arrays; does not touch the stats.
        Computed as the negation of the reference's rejection test |qf - mf| > limit, so a
        NaN label (which never satisfies it) is accepted, as in gate_candidate."""
        f = np.asarray(self.floor_labels)
        with np.errstate(invalid='ignore'):
            return ~(np.abs(f[np.asarray(query_idx)] - f[np.asarray(match_idx)]) > self._limit())

    def gate_candidates(self, candidates: List[Tuple[int, int, float]]) -> Tuple[List, List]:
        if len(candidates) == 0:
            return [], []
        qi = [c[0] for c in candidates]
        mi = [c[1] for c in candidates]
        f = self.floor_labels
        ok = self.decide(qi, mi)
        valid, rejected = [], []
        for (q, m, s), good in zip(candidates, ok):
            qf, mf = f[q], f[m]
            if good:
                valid.append(LoopClosureCandidate(q, m, s, qf, mf))
            else:
                rejected.append(LoopClosureCandidate(q, m, s, qf, mf, False, self._reason(qf, mf)))
        self.stats['total_candidates'] += len(candidates)
        self.stats['accepted'] += len(valid)
        self.stats['rejected_cross_floor'] += len(rejected)
        return valid, rejected

    def get_stats(self) -> Dict:
        total = self.stats['total_candidates']
        if total > 0:
            self.stats['acceptance_rate'] = self.stats['accepted'] / total
            self.stats['rejection_rate'] = 1 - self.stats['acceptance_rate']
        return self.stats

    def print_summary(self):
        st = self.get_stats()
        bar = "=" * 50
        print("\n" + bar + "\nLOOP CLOSURE GATING SUMMARY\n" + bar)
        print(f"Total candidates:      {st['total_candidates']}")
        print(f"Accepted:              {st['accepted']}")
        print(f"Rejected (cross-floor): {st['rejected_cross_floor']}")
        if st['total_candidates'] > 0:
            print(f"Acceptance rate:       {st['acceptance_rate']:.1%}")
            print(f"Perceptual aliasing prevented: {st['rejected_cross_floor']}")
        print(bar)


class ContextualPriorFactor:
    """GTSAM-style factor descriptions (plain dicts) from floor labels."""

    def __init__(self, floor_labels: np.ndarray):
        self.floor_labels = floor_labels

    def create_floor_constraint(self, pose_idx: int, floor_height: float = 3.0) -> Dict:
        floor = self.floor_labels[pose_idx]
        return {'type': 'floor_prior', 'pose_idx': pose_idx, 'floor': floor, 'expected_z': floor * floor_height,
                'noise_model': 'diagonal', 'sigma_z': 0.5}

    def create_elevator_transition_factor(self, pose_before: int, pose_after: int, direction: str,
                                          floor_height: float = 3.0) -> Dict:
        return {'type': 'elevator_transition', 'pose_before': pose_before, 'pose_after': pose_after,
                'expected_dz': floor_height if direction == 'up' else -floor_height, 'noise_model': 'diagonal',
                'sigma_dz': 0.3}


# the snippet text integrate_with_orbslam3 returns (loop_closure_gate.py:223-257), byte for
# byte: callers paste or diff it (tests/test_api_cpu.py against tests/golden/gate_snippet.json)
_ORBSLAM3_SNIPPET = """
// Add to LoopClosing.cc - DetectLoop() function
// After DBoW2 candidate retrieval, before geometric verification

bool LoopClosing::CheckFloorConsistency(KeyFrame* pKF, KeyFrame* pKFcandidate)
{
    // Get floor labels (stored in KeyFrame during tracking)
    int queryFloor = pKF->mnFloorLabel;
    int matchFloor = pKFcandidate->mnFloorLabel;
    
    // Strict mode: reject any cross-floor candidates
    if (queryFloor != matchFloor)
    {
        // Log rejected candidate for analysis
        VLOG(1) << "Loop closure rejected: Floor " << queryFloor 
                << " vs Floor " << matchFloor;
        return false;
    }
    
    return true;
}

// Modify DetectLoop() to call this before ComputeSim3()
vector<KeyFrame*> vpCandidateKFs = mpKeyFrameDB->DetectLoopCandidates(mpCurrentKF, minScore);

// Filter by floor consistency
vector<KeyFrame*> vpValidCandidates;
for(KeyFrame* pKF : vpCandidateKFs)
{
    if(CheckFloorConsistency(mpCurrentKF, pKF))
        vpValidCandidates.push_back(pKF);
}

// Continue with geometric verification on filtered candidates
"""


def integrate_with_orbslam3(floor_labels: np.ndarray, keyframe_times: np.ndarray) -> str:
    """C++ snippet (a string) for gating ORB-SLAM3's LoopClosing candidates by floor."""
    return _ORBSLAM3_SNIPPET
