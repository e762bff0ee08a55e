"""Oracle for the floor gate and the trajectory-proximity candidate generator
(test infrastructure only).

  * gate_decisions -- SemanticLoopClosureGate.gate_candidate(s) / get_stats
    (loop_closure_gate.py:60-134): diff = |floor[q] - floor[m]|; strict rejects
    diff > 0, non-strict rejects diff > 1; stats keys and rates as the reference.
  * proximity_candidates -- detect_loop_closure_candidates of the ORB-SLAM3 /
    LeGO-LOAM integrations (orb_slam3_integration.py:167-217,
    lego_loam_integration.py:121-157): pairs (i, j), i < j, |i - j| >= min_gap,
    ||p_i - p_j|| <= r (KDTree.query_ball_point is inclusive).  Returned sorted by
    (i, j); the KDTree emission order within a row is an artefact of the tree.
"""
import numpy as np


def gate_decisions(floor_labels, q, m, strict=True):
    f = np.asarray(floor_labels)
    qf, mf = f[np.asarray(q)], f[np.asarray(m)]
    diff = np.abs(qf - mf)
    valid = diff == 0 if strict else diff <= 1
    return valid, qf, mf


def gate_stats(valid):
    total = int(len(valid))
    acc = int(np.sum(valid))
    st = {'total_candidates': total, 'accepted': acc, 'rejected_cross_floor': total - acc, 'rejected_other': 0}
    if total > 0:
        st['acceptance_rate'] = acc / total
        st['rejection_rate'] = 1 - st['acceptance_rate']
    return st


def rejection_reason(qf, mf, strict=True):
    return (f"Cross-floor: {qf} vs {mf}" if strict else f"Floor diff > 1: {qf} vs {mf}")


def proximity_candidates(pos, radius=2.0, min_gap=100):
    """All (i, j) with i < j, j - i >= min_gap and ||p_i - p_j|| <= radius, sorted."""
    from scipy.spatial import cKDTree
    pos = np.asarray(pos, dtype=np.float64)
    pairs = cKDTree(pos).query_pairs(radius, output_type="ndarray")
    if len(pairs) == 0:
        return np.zeros((0, 2), np.int64)
    pairs = np.sort(pairs, axis=1)
    pairs = pairs[(pairs[:, 1] - pairs[:, 0]) >= min_gap]
    order = np.lexsort((pairs[:, 1], pairs[:, 0]))
    return pairs[order].astype(np.int64)
