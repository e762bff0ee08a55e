"""Device-resident all-keyframes retrieval: cosine kNN + time mask + threshold + floor gate.

Thin host wrapper over ``mlg_knn_gate`` (include/mlgate.h), which replaces
SemanticPlaceRecognition.find_loop_closures (place_recognition.py:851-911) and
BasePlaceRecognition.compute_all_pairwise_similarities (:179-190).
"""
import numpy as np

from . import _native

# k <= 32: fused scan; <= 256: per-lane lists; beyond: radix select in windows of 4096 ranks
# (knn.hip k_topk_large) -- no upper limit, as the reference's argsort()[:k] has none


def knn_gate(desc, t, floor, has_floor, min_gap, thr, k, gating, q0=0, Q=None, totals=None):
    """desc f32 [N, D], t f64 [N], floor i64 [N], has_floor u8 [N] -- all on the device.
    The threshold compares against float32 similarities in float32 (NumPy >= 2 / NEP 50
    semantics of the reference's ``similarities[j] < self.similarity_threshold``).

    Returns device tensors idx int32 [Q, k], sim f32 [Q, k], valid uint8 [Q, k], count int32 [Q].
    """
    if k < 1:
        raise ValueError(f"k must be >= 1 (got {k})")
    N = desc.shape[0]
    Q = N - q0 if Q is None else Q
    return _native.ops().knn_gate(desc, t, floor, has_floor, float(min_gap), float(thr), int(k), bool(gating),
                                  int(q0), int(Q), totals)


def pairwise_similarities(desc):
    """Device float32 N x N cosine similarity matrix (compute_all_pairwise_similarities)."""
    ops = _native.ops()
    xn = ops.row_normalize(desc)
    return ops.similarity(xn, xn)


def similarity(A, B):
    """Cosine similarities S[Q, N] between the rows of A [Q, D] and B [N, D] (device, float32)."""
    ops = _native.ops()
    return ops.similarity(ops.row_normalize(A), ops.row_normalize(B))


def flatten_matches(idx, sim, valid, count, q0=0):
    """Host flat arrays (q, m, sim, valid) in emission order from per-row device outputs."""
    idx, sim, valid, count = (x.cpu().numpy() for x in (idx, sim, valid, count))
    sel = np.arange(idx.shape[1])[None, :] < count[:, None]
    q = np.repeat(np.arange(q0, q0 + len(count)), count)
    return q, idx[sel].astype(np.int64), sim[sel], valid[sel].astype(bool)


def knn_query(db, qdesc, t_db, t_query, min_gap, k):
    """BasePlaceRecognition.query on the device: db f32 [N, D], qdesc f32 [Q, D], t_db f64 [N],
    t_query f64 [Q] (NaN = no timestamp).  Returns device idx int32 [Q, k], sim f32 [Q, k], count [Q]."""
    if k < 1:
        raise ValueError(f"k must be >= 1 (got {k})")
    return _native.ops().knn_query(db, qdesc, t_db, t_query, float(min_gap), int(k))


def xcorr_score(qf, mf):
    """CricaVPR.compute_cross_correlation_score on device float32 [n1, D] / [n2, D] -> device scalar."""
    return _native.ops().xcorr_score(qf.contiguous(), mf.contiguous())
