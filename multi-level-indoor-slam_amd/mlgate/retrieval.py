"""Device-resident all-keyframes retrieval: cosine kNN + time mask + threshold + floor gate.

Thin host wrapper over ``mlg_knn_gate`` (include/mlgate.h), which replaces
SemanticPlaceRecognition.find_loop_closures (place_recognition.py:851-911) and
BasePlaceRecognition.compute_all_pairwise_similarities (:179-190).
"""
import numpy as np
import torch

from . import _native

MAX_K = 256


class KnnWorkspace:
    """Cached device workspace (grows on demand) for mlg_knn_gate."""

    def __init__(self, device):
        self.device = device
        self.buf = None

    def get(self, nbytes):
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        return self.buf


_ws_cache = {}


def _workspace(device, nbytes):
    key = str(device)
    if key not in _ws_cache:
        _ws_cache[key] = KnnWorkspace(device)
    return _ws_cache[key].get(nbytes)


def knn_gate(desc, t, floor, has_floor, min_gap, thr, k, gating, q0=0, Q=None, totals=None):
    """desc f32 [N, D], t f64 [N], floor i64 [N], has_floor u8 [N] -- all on the device.

    Returns device tensors idx int32 [Q, k], sim f32 [Q, k], valid uint8 [Q, k], count int32 [Q].
    """
    if not 1 <= k <= MAX_K:
        raise ValueError(f"k must be in [1, {MAX_K}] (got {k})")
    N, D = desc.shape
    Q = N - q0 if Q is None else Q
    dev = desc.device
    L = _native.lib()
    nbytes = L.mlg_knn_workspace_bytes(N, D, Q)
    ws = _workspace(dev, nbytes)
    idx = torch.empty(Q, k, dtype=torch.int32, device=dev)
    sim = torch.empty(Q, k, dtype=torch.float32, device=dev)
    valid = torch.empty(Q, k, dtype=torch.uint8, device=dev)
    count = torch.empty(Q, dtype=torch.int32, device=dev)
    rc = L.mlg_knn_gate(_native.ptr(desc), N, D, _native.ptr(t), _native.ptr(floor), _native.ptr(has_floor),
                        float(min_gap), float(np.float32(thr)), int(k), int(bool(gating)), int(q0), int(Q),
                        _native.ptr(ws), ws.numel(), _native.ptr(idx), _native.ptr(sim), _native.ptr(valid),
                        _native.ptr(count), _native.ptr(totals) if totals is not None else None,
                        _native.stream_of(dev))
    _native.check(rc, "mlg_knn_gate")
    return idx, sim, valid, count


def pairwise_similarities(desc):
    """Device float32 N x N cosine similarity matrix (compute_all_pairwise_similarities)."""
    N, D = desc.shape
    dev = desc.device
    L = _native.lib()
    xn = torch.empty_like(desc)
    S = torch.empty(N, N, dtype=torch.float32, device=dev)
    st = _native.stream_of(dev)
    _native.check(L.mlg_row_normalize_f32(_native.ptr(desc), _native.ptr(xn), N, D, None, st), "normalize")
    _native.check(L.mlg_similarity(_native.ptr(xn), N, _native.ptr(xn), N, D, _native.ptr(S), st), "similarity")
    return S


def similarity(A, B):
    """Cosine similarities S[Q, N] between the rows of A [Q, D] and B [N, D] (device, float32)."""
    Q, D = A.shape
    N = B.shape[0]
    L = _native.lib()
    st = _native.stream_of(A.device)
    an, bn = torch.empty_like(A), torch.empty_like(B)
    S = torch.empty(Q, N, dtype=torch.float32, device=A.device)
    _native.check(L.mlg_row_normalize_f32(_native.ptr(A), _native.ptr(an), Q, D, None, st), "normalize")
    _native.check(L.mlg_row_normalize_f32(_native.ptr(B), _native.ptr(bn), N, D, None, st), "normalize")
    _native.check(L.mlg_similarity(_native.ptr(an), Q, _native.ptr(bn), N, D, _native.ptr(S), st), "similarity")
    return S


def flatten_matches(idx, sim, valid, count, q0=0):
    """Host flat arrays (q, m, sim, valid) in emission order from per-row device outputs."""
    idx, sim, valid, count = (x.cpu().numpy() for x in (idx, sim, valid, count))
    sel = np.arange(idx.shape[1])[None, :] < count[:, None]
    q = np.repeat(np.arange(q0, q0 + len(count)), count)
    return q, idx[sel].astype(np.int64), sim[sel], valid[sel].astype(bool)


def knn_query(db, qdesc, t_db, t_query, min_gap, k):
    """BasePlaceRecognition.query on the device: db f32 [N, D], qdesc f32 [Q, D], t_db f64 [N],
    t_query f64 [Q] (NaN = no timestamp).  Returns device idx int32 [Q, k], sim f32 [Q, k], count [Q]."""
    if not 1 <= k <= MAX_K:
        raise ValueError(f"k must be in [1, {MAX_K}] (got {k})")
    N, D = db.shape
    Q = qdesc.shape[0]
    dev = db.device
    L = _native.lib()
    ws = _workspace(dev, L.mlg_knn_workspace_bytes(N, D, Q))
    idx = torch.empty(Q, k, dtype=torch.int32, device=dev)
    sim = torch.empty(Q, k, dtype=torch.float32, device=dev)
    count = torch.empty(Q, dtype=torch.int32, device=dev)
    rc = L.mlg_knn_query(_native.ptr(db), N, D, _native.ptr(qdesc), Q, _native.ptr(t_db), _native.ptr(t_query),
                         float(min_gap), int(k), _native.ptr(ws), ws.numel(), _native.ptr(idx), _native.ptr(sim),
                         _native.ptr(count), _native.stream_of(dev))
    _native.check(rc, "mlg_knn_query")
    return idx, sim, count


def xcorr_score(qf, mf):
    """CricaVPR.compute_cross_correlation_score on device float32 [n1, D] / [n2, D] -> device scalar."""
    n1, D = qf.shape
    n2 = mf.shape[0]
    dev = qf.device
    L = _native.lib()
    ws = _workspace(dev, L.mlg_xcorr_workspace_bytes(n1, n2, D))
    out = torch.empty(1, dtype=torch.float32, device=dev)
    rc = L.mlg_xcorr_score(_native.ptr(qf), n1, _native.ptr(mf), n2, D, _native.ptr(ws), ws.numel(),
                           _native.ptr(out), _native.stream_of(dev))
    _native.check(rc, "mlg_xcorr_score")
    return out
