"""The full semantic gate on the GPU (mlgate.pipeline) against the fp32 oracle chain
(oracle/pipeline.py; golden outputs in tests/golden/gate_chain.npz, made by
tests/golden/make_gate_chain.py from the same seeded sequence).

Bar (north star: identical false-loop-closure rejection count, identical decisions):
  * floor labels from the IMU log: bit-exact;
  * descriptors: 1 - cos <= 1e-4 against the fp32 oracle;
  * retrieval: (a) bit-exact -- indices, emission order, is_valid, sims <= 4e-6 --
    against the oracle's find_loop_closures on the GPU's descriptors; (b) per query row
    the same (match, is_valid) set as the fp32 oracle chain (the fixture's sequence has
    every retrieval decision >= 5e-5 away from a flip);
  * verification: the cross-floor skip and is_valid of every pair identical to the fp32
    chain (SuperPoint + LightGlue fp32, OpenCV's RANSAC loop); inlier counts within
    3 % (at least 1) of the fp32 chain's (measured max 1.1 %: bf16 matches differ from fp32 ones);
  * floor gate verdicts and all four terms of the rejection count: identical.
Three configurations exercise every term: A (retrieval and verifier floor gating on),
B (retrieval gating off: the verifier skip engages), C (both off: aliased cross-floor
revisits pass verification and only the floor gate stops them).
"""
import json

import numpy as np
import pytest
import torch

from mlgate import synthetic
from mlgate.pipeline import DeviceGate, FullSemanticGate
from oracle import geometry as ogeo
from oracle import retrieval as oret

pytestmark = pytest.mark.gpu
CFG = {"A": (True, True), "B": (False, True), "C": (False, False)}


@pytest.fixture(scope="module")
def chain(golden_dir):
    g = dict(np.load(f"{golden_dir}/gate_chain.npz"))
    n, places, seed, k = (int(x) for x in g["params"])
    plan = tuple((int(f), float(p)) for f, p in g["plan"])
    seq = synthetic.make_sequence(n, places, seed, plan)
    g["seq"], g["frames"], g["imu"] = seq, synthetic.frames_host(seq), synthetic.imu_log(seq)
    g["k"], (g["thr"], g["gap"]) = k, (float(x) for x in g["thr_gap"])
    g["counts"] = json.loads(str(g["counts"]))
    g["pair_index"] = {tuple(p): i for i, p in enumerate(g["pairs"].tolist())}
    return g


@pytest.fixture(scope="module")
def reports(dev, chain):
    out = {}
    frames = torch.from_numpy(chain["frames"]).to(dev)
    for c, (rg, vg) in CFG.items():
        fg = FullSemanticGate(device=str(dev), k=chain["k"], similarity_threshold=chain["thr"],
                              min_time_gap=chain["gap"], retrieval_floor_gating=rg, verifier_floor_gating=vg)
        out[c] = (fg, fg.run(frames, chain["seq"].t, K=ogeo.ISEC_K, imu=chain["imu"]))
    return out


def test_floor_labels_and_descriptors(chain, reports):
    fg, rep = reports["A"]
    assert np.array_equal(rep.floor_labels, chain["labels"])
    D = np.stack([d.descriptor for d in fg.spr.vpr.descriptors]).astype(np.float64)
    R = chain["desc"].astype(np.float64)
    cos = np.sum(D * R, 1) / np.linalg.norm(D, axis=1) / np.linalg.norm(R, axis=1)
    assert np.max(1 - cos) <= 1e-4, np.max(1 - cos)


@pytest.mark.parametrize("cfg", list(CFG))
def test_retrieval_matches_oracle(chain, reports, cfg):
    fg, rep = reports[cfg]
    q = np.array([m.query_idx for m in rep.matches])
    mi = np.array([m.match_idx for m in rep.matches])
    sim = np.array([m.similarity for m in rep.matches], np.float32)
    val = np.array([m.is_valid for m in rep.matches])
    # (a) stage-anchored: the oracle's find_loop_closures on the GPU descriptors
    D = np.stack([d.descriptor for d in fg.spr.vpr.descriptors])
    lab = chain["labels"]
    oq, om, osim, ov = oret.find_loop_closures(D, chain["seq"].t, lab, np.ones(len(lab), np.uint8), chain["gap"],
                                               chain["thr"], chain["k"], CFG[cfg][0])
    assert np.array_equal(q, oq) and np.array_equal(mi, om) and np.array_equal(val, ov.astype(bool))
    assert np.max(np.abs(sim - osim)) <= 4e-6
    # (b) independent fp32 chain: the same (match, verdict) set per query row
    for r in np.unique(np.r_[q, chain[f"{cfg}_q"]]):
        got = {(int(a), bool(v)) for a, v in zip(mi[q == r], val[q == r])}
        sel = chain[f"{cfg}_q"] == r
        ref = {(int(a), bool(v)) for a, v in zip(chain[f"{cfg}_m"][sel], chain[f"{cfg}_valid"][sel])}
        assert got == ref, (r, got, ref)


@pytest.mark.parametrize("cfg", list(CFG))
def test_verification_and_gate_match_oracle(chain, reports, cfg):
    fg, rep = reports[cfg]
    assert len(rep.verified) == int(chain[f"{cfg}_valid"].sum())
    labels = chain["labels"]
    inl_got, inl_ref = [], []
    for m, r in zip(rep.verified, rep.results):
        skipped = CFG[cfg][1] and labels[m.query_idx] != labels[m.match_idx]
        if skipped:
            assert not r.is_valid and r.num_matches == 0
            continue
        i = chain["pair_index"][(m.query_idx, m.match_idx)]
        assert r.is_valid == bool(chain["pair_valid"][i]), (m.query_idx, m.match_idx, r, chain["pair_inliers"][i])
        if r.is_valid:
            inl_got.append(r.num_inliers)
            inl_ref.append(int(chain["pair_inliers"][i]))
    inl_got, inl_ref = np.array(inl_got), np.array(inl_ref)
    if len(inl_ref):
        rel = np.abs(inl_got - inl_ref) / inl_ref
        print(f"{cfg}: {len(inl_ref)} valid pairs, inlier |diff| / ref max {rel.max():.4f} mean {rel.mean():.4f}")
        # measured max 0.011 (profiles/r03ae_tolerances.log): bf16 matches vs the fp32 chain
        assert np.all(np.abs(inl_got - inl_ref) <= np.maximum(1, 0.03 * inl_ref)), list(zip(inl_got, inl_ref))
    # the gate on the geometrically valid pairs
    ok = [(m.query_idx, m.match_idx) for m, r in zip(rep.verified, rep.results) if r.is_valid]
    gv = chain[f"{cfg}_gate_valid"]
    assert len(ok) == len(gv)
    assert [c.is_valid for c in rep.accepted + rep.rejected] == [True] * len(rep.accepted) + [False] * len(
        rep.rejected)
    assert len(rep.accepted) == int(gv.sum()) and len(rep.rejected) == int((~gv).sum())
    # the four-term false-loop-closure rejection count
    assert rep.rejections.as_dict() == chain["counts"][cfg], (rep.rejections.as_dict(), chain["counts"][cfg])


def test_every_term_is_exercised(chain):
    c = chain["counts"]
    assert c["A"]["retrieval_floor_rejected"] > 0 and c["A"]["verifier_invalid"] > 0
    assert c["B"]["skipped_floor_mismatch"] > 0
    assert c["C"]["gate_rejected_cross_floor"] > 0


@pytest.mark.parametrize("cfg", list(CFG))
def test_device_gate_counts_equal_full_gate(dev, chain, reports, cfg):
    """bench.py's DeviceGate (device arrays, no objects) makes the same decisions."""
    _, rep = reports[cfg]
    frames = torch.from_numpy(chain["frames"]).to(dev)
    rg, vg = CFG[cfg]
    g = DeviceGate(frames, chain["seq"].t, chain["labels"], device=str(dev), k=chain["k"],
                   similarity_threshold=chain["thr"], min_time_gap=chain["gap"], retrieval_floor_gating=rg,
                   verifier_floor_gating=vg, K=ogeo.ISEC_K, vit_batch=64, lg_chunk=64)
    out = g.step()
    got = {k: out[k] for k in ("retrieval_floor_rejected", "skipped_floor_mismatch", "verifier_invalid",
                               "gate_rejected_cross_floor")}
    got["total"] = sum(got.values())
    assert got == rep.rejections.as_dict()
    assert out["matches"] == len(rep.matches) and out["accepted"] == len(rep.accepted)


@pytest.mark.parametrize("cfg", list(CFG))
def test_device_gate_unordered_matching_changes_nothing(dev, chain, cfg, monkeypatch):
    """LightGlue once per unordered pair (the default) vs once per ordered pair: the same
    counts and, PER ORDERED PAIR, the same match count, inlier count and decision in every
    configuration (LightGlue(b, a) is exactly swap(LightGlue(a, b)):
    test_lightglue_gpu.py::test_lightglue_swapped_pair_is_the_exact_swap)."""
    frames = torch.from_numpy(chain["frames"]).to(dev)
    rg, vg = CFG[cfg]
    outs, recs = {}, {}
    for dd in ("1", "0"):
        monkeypatch.setenv("MLGATE_LG_DEDUP", dd)
        g = DeviceGate(frames, chain["seq"].t, chain["labels"], device=str(dev), k=chain["k"],
                       similarity_threshold=chain["thr"], min_time_gap=chain["gap"], retrieval_floor_gating=rg,
                       verifier_floor_gating=vg, K=ogeo.ISEC_K, vit_batch=64, lg_chunk=64, record=True)
        outs[dd] = g.step()
        r = g.last_pair_results
        recs[dd] = {(int(x), int(y)): (int(n), int(i), bool(v))
                    for x, y, n, i, v in zip(r["a"], r["b"], r["matches"], r["inliers"], r["is_valid"])}
    a, b = dict(outs["1"]), dict(outs["0"])
    assert a.pop("pairs_matched_lightglue") <= b.pop("pairs_matched_lightglue")
    assert a == b
    assert recs["1"] == recs["0"]
    assert len(recs["1"]) == a["pairs_verified"] > 0


def test_superpoint_overlap_changes_nothing(dev, chain, monkeypatch):
    """SuperPoint of the keyframes past the first LightGlue chunk on a side stream under
    that chunk (MLGATE_SP_OVERLAP=1) vs every keyframe first (the default): the same counts
    and, per ordered pair, the same match count, inlier count and decision; several
    chunks, so the side-stream rows feed later chunks, and two steps, so a step starts
    from the previous step's tables."""
    frames = torch.from_numpy(chain["frames"]).to(dev)
    outs, recs = {}, {}
    for ov in ("1", "0"):
        monkeypatch.setenv("MLGATE_SP_OVERLAP", ov)
        g = DeviceGate(frames, chain["seq"].t, chain["labels"], device=str(dev), k=chain["k"],
                       similarity_threshold=chain["thr"], min_time_gap=chain["gap"], K=ogeo.ISEC_K,
                       vit_batch=64, lg_chunk=16, sp_batch=8, record=True)
        for _ in range(2):
            outs[ov] = g.step()
            r = g.last_pair_results
            recs[ov] = {(int(x), int(y)): (int(n), int(i), bool(v))
                        for x, y, n, i, v in zip(r["a"], r["b"], r["matches"], r["inliers"], r["is_valid"])}
    assert outs["1"] == outs["0"]
    assert recs["1"] == recs["0"] and len(recs["1"]) > 0


def test_orient_matches_is_the_swapped_call(dev):
    """mlg_lg_orient_matches: (i0, i1) -> (i1, i0) sorted by the new image0 index, scores
    carried along; unswapped rows copied."""
    from mlgate import _native
    rng = np.random.default_rng(3)
    R, K = 5, 300
    m = np.full((R, K, 2), -7, np.int32)
    sc = np.zeros((R, K), np.float32)
    n = rng.integers(0, K, R).astype(np.int32)
    for r in range(R):
        i0 = np.sort(rng.choice(K, n[r], replace=False))
        i1 = rng.choice(K, n[r], replace=False)
        m[r, :n[r], 0], m[r, :n[r], 1] = i0, i1
        sc[r, :n[r]] = rng.random(n[r])
    rows = np.array([0, 1, 1, 4, 2, 3], np.int32)
    swap = np.array([1, 0, 1, 1, 0, 1], np.uint8)
    T = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
    mo, so, no = _native.ops().lg_orient(T(m), T(sc), T(n), T(rows), T(swap))
    mo, so, no = mo.cpu().numpy(), so.cpu().numpy(), no.cpu().numpy()
    for p, (r, s_) in enumerate(zip(rows, swap)):
        k = n[r]
        assert no[p] == k
        if s_:
            o = np.argsort(m[r, :k, 1])
            assert np.array_equal(mo[p, :k, 0], m[r, :k, 1][o]) and np.array_equal(mo[p, :k, 1], m[r, :k, 0][o])
            assert np.array_equal(so[p, :k], sc[r, :k][o])
        else:
            assert np.array_equal(mo[p, :k], m[r, :k]) and np.array_equal(so[p, :k], sc[r, :k])


def test_ransac_inliers_equal_opencv_loop_on_gpu_matches(dev, chain, reports):
    """Stage-anchored RANSAC: on the GPU's own matches, the GPU inlier count equals that
    of OpenCV's sequential RANSAC loop restated in numpy (same cv::RNG sample stream)."""
    fg, rep = reports["A"]
    lg = fg.verifier.matcher
    frames = torch.from_numpy(chain["frames"]).to(dev)
    valid = [(m.query_idx, m.match_idx) for m, r in zip(rep.verified, rep.results) if r.is_valid][:2]
    invalid = [(m.query_idx, m.match_idx) for m, r in zip(rep.verified, rep.results)
               if not r.is_valid and r.num_matches >= 15][:1]
    pairs = valid + invalid
    matched = lg.detect_and_match_batch(frames, pairs)
    for (a, b), (k1, k2, _), r in zip(pairs, matched, [rep.results[[(m.query_idx, m.match_idx) for m in
                                                                    rep.verified].index(p)] for p in pairs]):
        _, mask, n_in = ogeo.cv_ransac(k1, k2, ogeo.ISEC_K, 3.0)
        # same sample stream and control flow; the two 5-point solvers' models differ in
        # the last bits, which can move a point sitting on the threshold (<= 0.3 %)
        assert abs(r.num_inliers - n_in) <= max(1, 0.003 * len(k1)), ((a, b), r.num_inliers, n_in)


def test_device_gate_float_and_missing_labels(dev, chain):
    """DeviceGate takes float labels with the reference's semantics: a non-integer floor,
    a NaN (never equal to anything -- retrieval floor check, verifier skip -- and never
    rejected by the gate's |df| > limit) -- the same four-term count as the drop-in
    FullSemanticGate on the same labels.  (None labels are accepted by retrieval and the
    verifier as the reference accepts them; the reference's gate cannot take them.)"""
    frames = torch.from_numpy(chain["frames"]).to(dev)
    lab = np.array([float(x) for x in chain["labels"]], np.float64)
    lab[3] = np.nan
    lab[lab == lab[0]] += 0.5
    for rg, vg in ((True, True), (False, True), (False, False)):
        fg = FullSemanticGate(device=str(dev), k=chain["k"], similarity_threshold=chain["thr"],
                              min_time_gap=chain["gap"], retrieval_floor_gating=rg, verifier_floor_gating=vg)
        rep = fg.run(frames, chain["seq"].t, K=ogeo.ISEC_K, floor_labels=lab)
        g = DeviceGate(frames, chain["seq"].t, lab, device=str(dev), k=chain["k"], similarity_threshold=chain["thr"],
                       min_time_gap=chain["gap"], retrieval_floor_gating=rg, verifier_floor_gating=vg,
                       K=ogeo.ISEC_K, vit_batch=64, lg_chunk=64)
        out = g.step()
        got = {k: out[k] for k in ("retrieval_floor_rejected", "skipped_floor_mismatch", "verifier_invalid",
                                   "gate_rejected_cross_floor")}
        got["total"] = sum(got.values())
        assert got == rep.rejections.as_dict(), (rg, vg, got, rep.rejections.as_dict())


def test_synthetic_frames_shard_equal_whole_sequence():
    """frames_device renders keyframe i from draw i of one seeded stream whichever frames
    are asked for, so each rank's shard is the same rows of the single-rank workload."""
    from mlgate import distributed as mdist
    seq = synthetic.make_sequence(24, 6, 0)
    dev = torch.device("cuda", 0)
    whole = synthetic.frames_device(seq, np.arange(24), dev, 64, 96)
    for world in (2, 3, 4):
        for r in range(world):
            lo, hi = mdist.shard(24, world, r)
            assert torch.equal(synthetic.frames_device(seq, np.arange(lo, hi), dev, 64, 96), whole[lo:hi])
    odd = np.array([17, 3, 9])
    assert torch.equal(synthetic.frames_device(seq, odd, dev, 64, 96), whole[torch.from_numpy(odd).to(dev)])
