"""Oracle for descriptor retrieval (test infrastructure only).

Restates, on the CPU, scripts/semantic_gating/place_recognition.py:
  * build_descriptor_matrix / compute_all_pairwise_similarities  (:173-190)
  * SemanticPlaceRecognition.find_loop_closures                   (:851-911)
  * SemanticPlaceRecognition.get_statistics                       (:913-933)
  * BasePlaceRecognition.query / _compute_similarity              (:117-171)

The similarity matrix is built with the same numpy calls the reference makes; the
O(N^2) per-row Python loop of the reference is restated in C (oracle.c:orc_knn_rows)
with one documented choice: np.argsort's default kind is unstable, so the order of
exactly-equal similarities is unpinned; the oracle (and the HIP kernel) order equal
similarities by descending index, i.e. a stable ascending argsort reversed.
"""
import numpy as np

from . import _lib


def normalize_rows(X):
    """desc / (||desc||_2 + 1e-8), float32 (place_recognition.py:186-187)."""
    X = np.asarray(X, dtype=np.float32)
    return X / (np.linalg.norm(X, axis=1, keepdims=True) + 1e-8)


def pairwise_similarities(X):
    """compute_all_pairwise_similarities (place_recognition.py:179-190)."""
    X = np.asarray(X)
    if X.size == 0:
        return np.array([])
    Xn = normalize_rows(X)
    return np.dot(Xn, Xn.T)


def find_loop_closures(X, t, floor, has_floor, min_gap=10.0, thr=0.5, k=10, gating=True, S=None):
    """Returns flat arrays (q, m, sim, valid) in the reference's emission order."""
    X = np.asarray(X, dtype=np.float32)
    n = X.shape[0]
    if n < 2:
        z = np.zeros(0, np.int64)
        return z, z, np.zeros(0, np.float32), np.zeros(0, np.uint8)
    if S is None:
        S = pairwise_similarities(X)
    idx, sim, valid, count = _lib.knn_rows(S, 0, t, floor, has_floor, min_gap, thr, k, gating)
    sel = np.arange(idx.shape[1])[None, :] < count[:, None]
    q = np.repeat(np.arange(n), count)
    return q.astype(np.int64), idx[sel].astype(np.int64), sim[sel], valid[sel]


def find_loop_closures_loop(X, t, floor_labels, min_gap=10.0, thr=0.5, k=10, gating=True, rows=None, S=None):
    """The reference's per-row Python loop itself (place_recognition.py:872-909), for timing
    the reference CPU path (bench.py cpu_baseline) and as a second restatement of the C
    loop: per query row a copy of the similarity row, the O(N) Python time mask, a full
    np.argsort, then threshold / floor check per top-k entry.  Ties: a stable ascending
    argsort reversed (the module's tie rule).  rows: the query rows to run (default all).
    Returns a list of (q, m, sim, is_valid)."""
    X = np.asarray(X, dtype=np.float32)
    n = X.shape[0]
    if n < 2:
        return []
    if S is None:
        S = pairwise_similarities(X)
    t = [float(v) for v in t]
    out = []
    for i in (range(n) if rows is None else rows):
        qt, qf = t[i], floor_labels[i]
        sims = S[i].copy()
        for j in range(n):
            if abs(t[j] - qt) < min_gap:
                sims[j] = -np.inf
        for j in np.argsort(sims, kind="stable")[::-1][:k]:
            if sims[j] < thr:
                continue
            mf = floor_labels[j]
            ok = True
            if gating and qf is not None and mf is not None:
                ok = qf == mf
            out.append((i, int(j), float(sims[j]), bool(ok)))
    return out


def statistics(sim, valid):
    """SemanticPlaceRecognition.get_statistics on flat arrays (place_recognition.py:913-933)."""
    n = len(sim)
    if n == 0:
        return {'total_matches': 0, 'valid_matches': 0, 'rejected_matches': 0, 'rejection_rate': 0.0}
    v = int(np.sum(valid))
    sims = [float(s) for s in sim]
    return {
        'total_matches': n,
        'valid_matches': v,
        'rejected_matches': n - v,
        'rejection_rate': (n - v) / n,
        'mean_similarity': np.mean(sims),
        'mean_valid_similarity': np.mean([s for s, ok in zip(sims, valid) if ok]) if v > 0 else 0.0,
    }


def query(db, qdesc, db_t, timestamp=None, k=5, min_gap=10.0):
    """BasePlaceRecognition.query given the query descriptor (place_recognition.py:117-163).

    Returns (match_idx, similarity); ties ordered by descending index (see module doc).
    """
    db = np.asarray(db, dtype=np.float32)
    if len(db) == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.float32)
    q = np.asarray(qdesc, dtype=np.float32)
    qn = q / (np.linalg.norm(q) + 1e-8)
    dbn = db / (np.linalg.norm(db, axis=1, keepdims=True) + 1e-8)
    s = np.dot(dbn, qn)
    if timestamp is not None:
        s[np.abs(np.asarray(db_t) - timestamp) < min_gap] = -np.inf
    order = np.argsort(s, kind="stable")[::-1][:k]
    order = order[s[order] > -np.inf]
    return order.astype(np.int64), s[order]
