"""Pin the CPU oracle against the reference's own outputs (golden vectors captured by
tests/golden/make_goldens.py) and the published gate counts.  CPU only."""
import glob
import json
import os

import numpy as np
import pytest

from oracle import _lib, floors, gate, retrieval, xcorr

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "knn_*.npz"))), ids=os.path.basename)
def test_oracle_find_loop_closures(path):
    g = dict(np.load(path, allow_pickle=False))
    k, thr, gap, gating = g["params"]
    q, m, sim, valid = retrieval.find_loop_closures(g["desc"].astype(np.float32), g["t"], g["floor"],
                                                    g["has_floor"], gap, thr, int(k), bool(gating))
    assert np.array_equal(q, g["q"]) and np.array_equal(m, g["m"])
    assert np.array_equal(valid.astype(bool), g["valid"].astype(bool))
    assert np.array_equal(sim.astype(np.float64), g["sim"])  # same numpy calls -> bit-identical
    st = retrieval.statistics(sim, valid)
    ref = json.loads(str(g["stats"]))
    assert set(st) == set(ref)
    for key in ref:
        assert st[key] == pytest.approx(ref[key], rel=0, abs=0), key


def test_oracle_norms_bit_exact_vs_numpy():
    rng = np.random.default_rng(0)
    for d in (7, 128, 768, 4096, 8448, 10752, 49152):
        X = rng.standard_normal((16, d)).astype(np.float32) * 3
        assert np.array_equal(_lib.row_norms_f32(X), np.linalg.norm(X, axis=1))


def test_oracle_pairwise():
    g = load("pairwise.npz")
    S = retrieval.pairwise_similarities(g["desc"].astype(np.float32))
    assert np.array_equal(S, g["S"])
    assert int(g["empty_size"]) == retrieval.pairwise_similarities(np.zeros((0, 768), np.float32)).size


def test_oracle_query():
    g = load("query.npz")
    for tag, ts, k, gap in (("a", 20.0, 5, 10.0), ("b", None, 5, 10.0), ("c", 100.0, 12, 30.0)):
        m, s = retrieval.query(g["desc"].astype(np.float32), g["qdesc"], g["t"], ts, k, gap)
        assert np.array_equal(m, g[f"{tag}_m"])
        assert np.array_equal(s.astype(np.float64), g[f"{tag}_sim"])


def test_oracle_xcorr():
    g = load("xcorr.npz")
    feats = g["feats"].astype(np.float32)
    for (a, b), ref in zip(g["pairs"], g["scores"]):
        assert xcorr.xcorr_score(feats[a], feats[b]) == ref
    assert xcorr.xcorr_score(feats[0][0], feats[1][0]) == float(g["s2d"])
    cache = {i: feats[i] for i in range(5)}
    cands = [(int(j), float(s)) for j, s in g["cands"]]
    rr = xcorr.rerank(cache, 0, cands, top_k=4)
    assert np.allclose(np.array(rr), g["rr"], rtol=0, atol=0)
    assert np.allclose(np.array(xcorr.rerank(cache, 5, cands, top_k=3)), g["rr_nocache"])


def test_oracle_gate():
    with open(os.path.join(GOLD, "gate.json")) as f:
        G = json.load(f)
    labels = np.zeros(10000, dtype=int)
    for a, b, fl in G["labels_blocks"]:
        labels[a:b] = fl
    for key, case in G.items():
        if not isinstance(case, dict) or "candidates" not in case:
            continue
        strict = key.endswith("strict")
        c = np.array([x[:2] for x in case["candidates"]], dtype=np.int64)
        valid, qf, mf = gate.gate_decisions(labels, c[:, 0], c[:, 1], strict)
        got_v = [[int(a), int(b)] for (a, b), ok in zip(c, valid) if ok]
        assert got_v == [v[:2] for v in case["valid"]]
        got_r = [[int(a), int(b), gate.rejection_reason(int(x), int(y), strict)]
                 for (a, b), ok, x, y in zip(c, valid, qf, mf) if not ok]
        assert got_r == case["rejected"]
        st = gate.gate_stats(valid)
        assert st == pytest.approx(case["stats"])


def test_oracle_imu_floors():
    g = load("imu.npz")
    ev = floors.detect_events(g["t"], g["ax"], g["ay"], g["az"])
    arr = np.array([[e[0], e[1], e[2], e[4], e[5], e[6]] for e in ev], np.float64).reshape(-1, 6)
    assert np.array_equal(arr, g["events"])
    assert [e[3] for e in ev] == list(g["directions"])
    assert np.array_equal(floors.assign_labels(g["traj"], ev, 5), g["labels"])


@pytest.mark.parametrize("system,counts", [("lego_loam", (87044, 21477, 65567)),
                                           ("orb_slam3", (5110618, 1498091, 3612527))])
def test_oracle_trajectory_gate_counts(system, counts):
    """The published gate counts (results/semantic_gating/*_semantic_analysis.txt:20-23)."""
    g = load(f"traj_{system}.npz")
    pairs = gate.proximity_candidates(g["pos"], 2.0, 100)
    valid, _, _ = gate.gate_decisions(g["floor"], pairs[:, 0], pairs[:, 1], True)
    total, same = len(pairs), int(valid.sum())
    assert (total, same, total - same) == counts == (int(g["total"]), int(g["same"]), int(g["cross"]))
    n = len(g["pos"])
    key = np.sort(pairs[:, 0] * n + pairs[:, 1])
    assert int(key.sum()) % (1 << 64) == int(g["pair_key_sum"])


def test_oracle_resize_identity_and_ramps():
    """Resize restatement sanity: identity size is exact; constant images stay constant."""
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (48, 64, 3), dtype=np.uint8)
    assert np.array_equal(_lib.resize_linear_u8(img, 48, 64), img)
    const = np.full((480, 640, 3), 173, np.uint8)
    assert np.all(_lib.resize_linear_u8(const, 322, 322) == 173)
    assert _lib.lib().orc_resize_vec_end(966) == 960


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "knn_*.npz")))[:4], ids=os.path.basename)
def test_oracle_python_loop_restatement(path):
    """retrieval.find_loop_closures_loop (the reference's per-row Python loop, timed as the
    reference CPU path by bench.py's cpu_baseline) equals the reference's golden output."""
    g = dict(np.load(path, allow_pickle=False))
    k, thr, gap, gating = g["params"]
    labels = [int(f) if h else None for f, h in zip(g["floor"], g["has_floor"])]
    out = retrieval.find_loop_closures_loop(g["desc"].astype(np.float32), g["t"], labels, gap, thr, int(k),
                                            bool(gating))
    assert [o[0] for o in out] == g["q"].tolist() and [o[1] for o in out] == g["m"].tolist()
    assert [o[3] for o in out] == g["valid"].astype(bool).tolist()
    assert np.array_equal(np.array([o[2] for o in out]), g["sim"])
