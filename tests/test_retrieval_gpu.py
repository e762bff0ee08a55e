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
