"""Trajectory-proximity candidates + floor gate on the GPU (proximity.hip via the C ABI).

Pinned by the reference's published gate counts on its committed trajectories
(results/semantic_gating/{lego_loam,orb_slam3}_semantic_analysis.txt:20-23, captured
with the candidate-set digest by tests/golden/make_goldens.py) and checked pair by pair
against the oracle (oracle/gate.py) on seeded cases that put points exactly on the
radius.  Pair sets, order and verdicts are bit-exact; distances within 1 ulp-ish.
"""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from mlgate import proximity
from oracle import gate as ogate

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


@pytest.mark.parametrize("system", ["lego_loam", "orb_slam3"])
def test_trajectory_gate_golden_counts(dev, system):
    g = load(f"traj_{system}.npz")
    tg = proximity.TrajectoryLoopClosureGate(g["pos"], g["floor"], device=str(dev))
    cands = tg.detect_loop_closure_candidates(2.0, 100)
    a = tg.apply_floor_gating(cands, strict_mode=True)
    assert (a.total_candidates, a.same_floor_candidates, a.cross_floor_candidates) == (
        int(g["total"]), int(g["same"]), int(g["cross"]))
    n = len(g["pos"])
    key = cands.pairs[:, 0] * n + cands.pairs[:, 1]
    assert np.all(np.diff(key) > 0), "pairs must come out in (i, j) order"
    assert hashlib.sha256(key.astype("<i8").tobytes()).hexdigest() == str(g["pair_sha256"])
    assert int(key.sum()) % (1 << 64) == int(g["pair_key_sum"])
    ref_stats = json.loads(str(g["gate_stats"]))
    st = tg.loop_gate.get_stats()
    assert set(st) == set(ref_stats)
    for k, v in ref_stats.items():
        assert st[k] == pytest.approx(v, rel=0, abs=1e-15), k
    # the reference's first cross-floor examples are in its cross set
    cross = {(int(i), int(j)) for i, j, _, _ in a.cross_floor_pairs[:200000]}
    for i, j in g["first_cross"]:
        assert (int(i), int(j)) in cross
    # distances: float64 norm of the difference
    d_ref = np.linalg.norm(g["pos"][cands.pairs[:, 0]] - g["pos"][cands.pairs[:, 1]], axis=1)
    np.testing.assert_allclose(cands.dist, d_ref, rtol=1e-14, atol=0)


def _boundary_case(seed, n):
    """Integer lattice positions: many pairs at exactly r = 2 (and sqrt(2), sqrt(3) ...)."""
    rng = np.random.default_rng(seed)
    walk = np.cumsum(rng.integers(-1, 2, (n, 3)), axis=0).astype(np.float64)
    walk[:, 2] = rng.integers(0, 3, n)  # a few "floors" of height
    floor = np.repeat(rng.integers(0, 4, n // 50 + 1), 50)[:n].astype(np.int64)
    return walk, floor


@pytest.mark.parametrize("seed,n,r,gap,strict", [(0, 3000, 2.0, 100, True), (1, 2500, 1.5, 10, False),
                                                 (2, 4100, 2.0, 1, True), (3, 700, 0.0, 5, True),
                                                 (4, 2049, 3.0, 2048, False)])
def test_proximity_matches_oracle(dev, seed, n, r, gap, strict):
    pos, floor = _boundary_case(seed, n)
    c = proximity.detect_loop_closure_candidates(pos, r, gap, floor, strict, device=str(dev))
    ref = ogate.proximity_candidates(pos, r, gap)
    assert np.array_equal(c.pairs, ref)
    v, _, _ = ogate.gate_decisions(floor, ref[:, 0], ref[:, 1], strict)
    assert np.array_equal(c.valid, v)
    assert c.accepted == int(v.sum())
    np.testing.assert_allclose(c.dist, np.linalg.norm(pos[ref[:, 0]] - pos[ref[:, 1]], axis=1), rtol=1e-15)


def test_proximity_row_ranges_concatenate(dev):
    pos, floor = _boundary_case(7, 5000)
    p = torch.from_numpy(pos).to(dev)
    f = torch.from_numpy(floor).to(dev)
    full = proximity.proximity_candidates_device(p, f, 2.0, 50)
    parts = [proximity.proximity_candidates_device(p, f, 2.0, 50, row0=a, nrows=b - a)
             for a, b in ((0, 1), (1, 1777), (1777, 4096), (4096, 5000))]
    for k in range(3):
        assert torch.equal(full[k], torch.cat([q[k] for q in parts]))
    assert full[3] == sum(q[3] for q in parts) and full[4] == sum(q[4] for q in parts)


def test_proximity_edges(dev):
    for n in (0, 1, 2):
        c = proximity.detect_loop_closure_candidates(np.zeros((n, 3)), 2.0, 1, np.zeros(n, np.int64),
                                                     device=str(dev))
        assert len(c) == (1 if n == 2 else 0)
    c = proximity.detect_loop_closure_candidates(np.zeros((50, 3)), 2.0, 100, device=str(dev))
    assert len(c) == 0 and c.to_list() == []
    with pytest.raises(ValueError):
        proximity.detect_loop_closure_candidates(np.zeros((70000, 3)), 2.0, 100, device=str(dev))
    with pytest.raises(ValueError):
        proximity.detect_loop_closure_candidates(np.zeros((10, 3)), 2.0, 0, device=str(dev))
