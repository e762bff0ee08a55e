"""Retrieval + gate parity on the GPU against golden vectors captured from the reference
(tests/golden/make_goldens.py).  Indices, emission order and gate decisions must be
bit-exact; similarities agree to SIM_TOL (the reference's OpenBLAS SGEMM and the f32
MFMA differ only in summation order)."""
import glob
import json
import os

import numpy as np
import pytest
import torch

from mlgate import retrieval

pytestmark = pytest.mark.gpu

# float32 dot products of unit vectors over D = 768..4096 terms: two summation orders
# (OpenBLAS SGEMM vs the f32 MFMA chain) differ by up to ~sqrt(D) * 2^-24 * few.
SIM_TOL = 4e-6


def load(path):
    return dict(np.load(path, allow_pickle=False))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "knn_*.npz"))),
                         ids=lambda p: os.path.basename(p))
def test_find_loop_closures_golden(dev, path):
    g = load(path)
    k, thr, gap, gating = g["params"]
    k, gating = int(k), bool(gating)
    desc = torch.from_numpy(g["desc"].astype(np.float32)).to(dev)
    t = torch.from_numpy(g["t"]).to(dev)
    fl = torch.from_numpy(g["floor"]).to(dev)
    hf = torch.from_numpy(g["has_floor"]).to(dev)
    totals = torch.zeros(2, dtype=torch.int64, device=dev)
    out = retrieval.knn_gate(desc, t, fl, hf, gap, thr, k, gating, totals=totals)
    q, m, sim, valid = retrieval.flatten_matches(*out)
    assert np.array_equal(q, g["q"])
    assert np.array_equal(m, g["m"])
    assert np.array_equal(valid, g["valid"].astype(bool))
    assert np.max(np.abs(sim.astype(np.float64) - g["sim"]), initial=0.0) <= SIM_TOL
    tv, tr = totals.cpu().tolist()
    assert tv == int(g["valid"].sum()) and tr == len(g["valid"]) - int(g["valid"].sum())


def test_pairwise_golden(dev):
    g = load(os.path.join(os.path.dirname(__file__), "golden", "pairwise.npz"))
    S = retrieval.pairwise_similarities(torch.from_numpy(g["desc"].astype(np.float32)).to(dev)).cpu().numpy()
    assert S.shape == g["S"].shape
    assert np.max(np.abs(S - g["S"])) <= SIM_TOL


def test_query_golden(dev):
    g = load(os.path.join(os.path.dirname(__file__), "golden", "query.npz"))
    db = torch.from_numpy(g["desc"].astype(np.float32)).to(dev)
    tdb = torch.from_numpy(g["t"]).to(dev)
    qd = torch.from_numpy(g["qdesc"][None].astype(np.float32)).to(dev)
    for tag, ts, k, gap in (("a", 20.0, 5, 10.0), ("b", None, 5, 10.0), ("c", 100.0, 12, 30.0)):
        tq = torch.tensor([np.nan if ts is None else ts], dtype=torch.float64, device=dev)
        idx, sim, count = retrieval.knn_query(db, qd, tdb, tq, gap, k)
        c = int(count[0])
        assert np.array_equal(idx[0, :c].cpu().numpy(), g[f"{tag}_m"])
        assert np.max(np.abs(sim[0, :c].cpu().numpy() - g[f"{tag}_sim"]), initial=0) <= SIM_TOL


def test_xcorr_golden(dev):
    g = load(os.path.join(os.path.dirname(__file__), "golden", "xcorr.npz"))
    feats = torch.from_numpy(g["feats"].astype(np.float32)).to(dev)
    for (a, b), ref in zip(g["pairs"], g["scores"]):
        s = retrieval.xcorr_score(feats[a, 0], feats[b, 0]).item()
        assert abs(s - ref) < 1e-5, (a, b, s, ref)


def test_large_n_self_consistency(dev):
    """N = 5000 (the configs[1] size): GPU == oracle on the same similarity matrix."""
    from oracle import _lib
    rng = np.random.default_rng(0)
    n, d = 5000, 768
    centres = rng.standard_normal((400, d)).astype(np.float32)
    X = (centres[rng.integers(0, 400, n)] + 0.8 * rng.standard_normal((n, d)).astype(np.float32))
    t = np.arange(n) * 0.765
    fl = np.repeat(np.array([5, 1, 4, 2]), [2275, 665, 680, 1380]).astype(np.int64)
    hf = np.ones(n, np.uint8)
    dX = torch.from_numpy(X).to(dev)
    out = retrieval.knn_gate(dX, torch.from_numpy(t).to(dev), torch.from_numpy(fl).to(dev),
                             torch.from_numpy(hf).to(dev), 10.0, 0.5, 10, True)
    q, m, sim, valid = retrieval.flatten_matches(*out)
    S = retrieval.pairwise_similarities(dX).cpu().numpy()  # the same matrix the kernel ranked
    idx, osim, ovalid, count = _lib.knn_rows(S, 0, t, fl, hf, 10.0, 0.5, 10, True)
    sel = np.arange(10)[None, :] < count[:, None]
    assert np.array_equal(m, idx[sel]) and np.array_equal(sim, osim[sel])
    assert np.array_equal(valid, ovalid[sel].astype(bool))
    assert len(m) > 1000


def _clustered(n, d=768, seed=0):
    rng = np.random.default_rng(seed)
    centres = rng.standard_normal((max(2, n // 12), d)).astype(np.float32)
    X = centres[rng.integers(0, len(centres), n)] + 0.8 * rng.standard_normal((n, d)).astype(np.float32)
    t = np.arange(n) * 0.765
    fl = rng.integers(1, 5, n).astype(np.int64)
    return X, t, fl, np.ones(n, np.uint8)


def _gate(dev, X, t, fl, hf, k, q0=0, Q=None, thr=0.5, gating=True):
    args = [torch.from_numpy(a).to(dev) for a in (X, t, fl, hf)]
    return retrieval.knn_gate(*args, 10.0, thr, k, gating, q0=q0, Q=Q)


def test_fused_scan_equals_materialised_path(dev):
    """k <= 32 runs the fused scan (S streamed through LDS, never stored); k > 32 the
    materialised S + per-row top-k.  The top-20 of the k = 40 run must equal the
    fused k = 20 run bit for bit (same similarity bits, same order, same verdicts)."""
    X, t, fl, hf = _clustered(3000, seed=1)
    i20, s20, v20, c20 = (a.cpu().numpy() for a in _gate(dev, X, t, fl, hf, 20, thr=0.3))
    i40, s40, v40, c40 = (a.cpu().numpy() for a in _gate(dev, X, t, fl, hf, 40, thr=0.3))
    assert np.array_equal(c20, np.minimum(c40, 20))
    assert c20.sum() > 20000
    for r in range(len(c20)):
        n = c20[r]
        assert np.array_equal(i20[r, :n], i40[r, :n]) and np.array_equal(s20[r, :n], s40[r, :n])
        assert np.array_equal(v20[r, :n], v40[r, :n])


@pytest.mark.parametrize("k", [10, 40])
def test_row_split_concatenates(dev, k):
    """Rank r > 0 of the multi-GPU path gates rows [q0, q0 + Q): the row ranges of a split
    concatenate to the full run, for the fused (k = 10) and materialised (k = 40) paths."""
    X, t, fl, hf = _clustered(1500, seed=2)
    full = retrieval.flatten_matches(*_gate(dev, X, t, fl, hf, k))
    parts = [retrieval.flatten_matches(*_gate(dev, X, t, fl, hf, k, q0=a, Q=b - a), q0=a)
             for a, b in ((0, 611), (611, 1100), (1100, 1500))]
    for i in range(4):
        assert np.array_equal(full[i], np.concatenate([p[i] for p in parts]))


def test_large_n_without_similarity_matrix(dev):
    """N = 19,163 (the ORB-SLAM3 frame count): the fused scan needs no
    [N, N] matrix (1.47 GB); peak device memory stays far below it, and sampled rows
    equal the oracle's ranking of the same similarity rows."""
    from oracle import _lib
    n = 19163
    X, t, fl, hf = _clustered(n, seed=3)
    dX = torch.from_numpy(X).to(dev)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(dev)
    base = torch.cuda.memory_allocated(dev)
    out = _gate(dev, X, t, fl, hf, 10)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated(dev) - base
    assert peak < 200 * 2 ** 20, peak  # normalised rows (59 MB) + partial lists, no S
    idx, sim, valid, count = (a.cpu().numpy() for a in out)
    rows = np.arange(0, n, 997)
    S = retrieval.similarity(dX[torch.from_numpy(rows).to(dev)], dX).cpu().numpy()
    for j, r in enumerate(rows):
        oi, osim, ov, oc = _lib.knn_rows(S[j:j + 1], int(r), t, fl, hf, 10.0, 0.5, 10, True)
        c = count[r]
        assert c == oc[0] and np.array_equal(idx[r, :c], oi[0, :c]) and np.array_equal(sim[r, :c], osim[0, :c])
        assert np.array_equal(valid[r, :c].astype(bool), ov[0, :c].astype(bool))


@pytest.mark.parametrize("k", [300, 1000, 4096])
@pytest.mark.parametrize("gating", [True, False])
def test_large_k_radix_select(dev, k, gating):
    """256 < k <= 4096 (k_topk_large: radix select + LDS sort) against the oracle's
    per-row loop on the same similarity matrix: indices, order, validity bit-exact."""
    from oracle import retrieval as oret
    rng = np.random.default_rng(k)
    n, d = 1500, 64
    X = rng.standard_normal((n, d)).astype(np.float32)
    t = np.arange(n, dtype=np.float64) * 0.7
    fl = rng.integers(0, 4, n).astype(np.int64)
    hf = (rng.random(n) > 0.1).astype(np.uint8)
    thr = -0.05 if k != 1000 else 0.02
    Xd = torch.from_numpy(X).to(dev)
    S = retrieval.pairwise_similarities(Xd).cpu().numpy()
    out = retrieval.knn_gate(Xd, torch.from_numpy(t).to(dev), torch.from_numpy(fl).to(dev),
                             torch.from_numpy(hf).to(dev), 10.0, thr, k, gating)
    q, m, sim, valid = retrieval.flatten_matches(*out)
    rq, rm, rs, rv = oret.find_loop_closures(X, t, fl, hf, 10.0, thr, k, gating, S=S)
    assert np.array_equal(q, rq) and np.array_equal(m, rm)
    assert np.array_equal(valid, rv.astype(bool))
    assert np.array_equal(sim, rs)


@pytest.mark.parametrize("k", [300, 1000])
def test_query_large_k(dev, k):
    """query() with k > 256 (k_topk_large): the first 256 entries equal the k = 256 path
    bit for bit, the sorted similarities match the oracle's within SIM_TOL, the order is
    (similarity desc, index desc), and the count is every unmasked entry up to k."""
    from oracle import retrieval as oret
    rng = np.random.default_rng(7 + k)
    n = 1500
    db = rng.standard_normal((n, 64)).astype(np.float32)
    q = rng.standard_normal(64).astype(np.float32)
    t = np.arange(n, dtype=np.float64) * 0.7
    ts, gap = 300.0, 10.0
    dbd = torch.from_numpy(db).to(dev)
    tdb = torch.from_numpy(t).to(dev)
    qd = torch.from_numpy(q[None]).to(dev)
    tq = torch.tensor([ts], dtype=torch.float64, device=dev)
    idx, sim, cnt = retrieval.knn_query(dbd, qd, tdb, tq, gap, k)
    i2, s2, c2 = retrieval.knn_query(dbd, qd, tdb, tq, gap, 256)
    c = int(cnt[0])
    idx, sim = idx[0, :c].cpu().numpy(), sim[0, :c].cpu().numpy()
    ro, rs = oret.query(db, q, t, ts, k, gap)
    assert c == len(ro) == min(k, int((np.abs(t - ts) >= gap).sum()))
    assert np.array_equal(idx[:256], i2[0, :256].cpu().numpy()) and np.array_equal(sim[:256], s2[0, :256].cpu().numpy())
    assert np.max(np.abs(sim - rs)) <= SIM_TOL
    assert np.all((sim[:-1] > sim[1:]) | ((sim[:-1] == sim[1:]) & (idx[:-1] > idx[1:])))
    assert len(set(idx.tolist())) == c and np.all(np.abs(t[idx] - ts) >= gap)


@pytest.mark.parametrize("L", [528, 200])
def test_xcorr_batch_equals_single_pairs(dev, L):
    """mlg_xcorr_batch (one pass over all (query, candidate) pairs, no [L, L] matrices)
    gives every pair exactly the single-pair mlg_xcorr_score bits; plus the golden pairs."""
    from mlgate import _native
    rng = np.random.default_rng(L)
    F, D = 7, 768
    feats = torch.from_numpy(rng.standard_normal((F, L, D)).astype(np.float32)).to(dev)
    qa = np.array([0, 0, 1, 3, 6, 2, 5, 4], np.int32)
    qb = np.array([1, 2, 0, 3, 5, 6, 0, 4], np.int32)
    got = _native.ops().xcorr_batch(feats, torch.from_numpy(qa).to(dev), torch.from_numpy(qb).to(dev)).cpu().numpy()
    for p, (a, b) in enumerate(zip(qa, qb)):
        ref = retrieval.xcorr_score(feats[a], feats[b]).item()
        assert np.float32(got[p]).tobytes() == np.float32(ref).tobytes(), (p, got[p], ref)
    g = load(os.path.join(os.path.dirname(__file__), "golden", "xcorr.npz"))
    gf = torch.from_numpy(g["feats"].astype(np.float32)[:, 0]).to(dev)
    pr = g["pairs"].astype(np.int32)
    sc = _native.ops().xcorr_batch(gf, torch.from_numpy(pr[:, 0].copy()).to(dev),
                                   torch.from_numpy(pr[:, 1].copy()).to(dev)).cpu().numpy()
    assert np.max(np.abs(sc - g["scores"])) < 1e-5


@pytest.mark.parametrize("k,thr", [(5000, -1.1), (20000, -1.1), (9000, -0.02)])
def test_k_beyond_4096_windows(dev, k, thr):
    """k > 4096 with N > 4096 (the reference's argsort()[:k] has no limit; k > N returns
    every candidate): k_topk_large emits its ranks in windows of 4096 -- indices, order,
    validity and similarities bit-exact against the oracle's per-row loop on the same S,
    including a threshold that stops emission inside a window."""
    from oracle import _lib
    rng = np.random.default_rng(k)
    n, d, q0, Q = 9000, 32, 4000, 64
    X = rng.standard_normal((n, d)).astype(np.float32)
    t = np.arange(n, dtype=np.float64) * 0.7
    fl = rng.integers(0, 4, n).astype(np.int64)
    hf = (rng.random(n) > 0.1).astype(np.uint8)
    Xd = torch.from_numpy(X).to(dev)
    out = retrieval.knn_gate(Xd, torch.from_numpy(t).to(dev), torch.from_numpy(fl).to(dev),
                             torch.from_numpy(hf).to(dev), 10.0, thr, k, True, q0=q0, Q=Q)
    idx, sim, valid, count = (x.cpu().numpy() for x in out)
    S = retrieval.pairwise_similarities(Xd)[q0:q0 + Q].cpu().numpy()
    ri, rs, rv, rc = _lib.knn_rows(S, q0, t, fl, hf, 10.0, thr, k, True)
    assert np.array_equal(count, rc) and count.max() > 4096
    for r in range(Q):
        c = int(count[r])
        assert np.array_equal(idx[r, :c], ri[r, :c]) and np.array_equal(sim[r, :c], rs[r, :c])
        assert np.array_equal(valid[r, :c].astype(bool), rv[r, :c].astype(bool))


def test_xcorr_batch_beyond_one_grid_slice(dev):
    """More pairs than one k_xcorr_tiles launch takes (slices of 16384; a bench step's
    rerank sends every (query, candidate) pair, ~100k): every pair still gets the
    single-pair bits, and the scores do not depend on where the slices fall."""
    from mlgate import _native
    rng = np.random.default_rng(5)
    F, L, D, P = 9, 40, 64, 70_001
    feats = torch.from_numpy(rng.standard_normal((F, L, D)).astype(np.float32)).to(dev)
    qa = rng.integers(0, F, P).astype(np.int32)
    qb = rng.integers(0, F, P).astype(np.int32)
    got = _native.ops().xcorr_batch(feats, torch.from_numpy(qa).to(dev), torch.from_numpy(qb).to(dev)).cpu().numpy()
    table = {(a, b): retrieval.xcorr_score(feats[a], feats[b]).item() for a in range(F) for b in range(F)}
    want = np.array([table[(a, b)] for a, b in zip(qa.tolist(), qb.tolist())], np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
