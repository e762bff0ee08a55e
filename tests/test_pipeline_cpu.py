"""CPU checks of the full-gate fixture and the pipeline's host logic.

  * the fixture (tests/golden/gate_chain.npz) is reproduced by the oracle chain from its
    own inputs: IMU floor labels, find_loop_closures on the stored fp32 descriptors, the
    skip rule, the floor gate and the four-term count (the per-pair fp32 verification
    verdicts are taken from the fixture; one pair is recomputed end to end);
  * the product's IMU path (mlgate.floors) gives the oracle's labels on that log;
  * OpenCV's RANSAC control flow restated in the oracle (cv::RNG stream, update rule);
  * host-side label semantics of the drop-ins (floor codes, NaN gate verdicts, k limit).
"""
import json

import numpy as np
import pytest

from mlgate import synthetic
from mlgate.gate import SemanticLoopClosureGate
from mlgate.pipeline import floor_labels_from_imu
from mlgate.vpr import PlaceDescriptor, SemanticPlaceRecognition, floor_codes
from oracle import geometry as ogeo
from oracle import pipeline as opipe

CFG = {"A": (True, True), "B": (False, True), "C": (False, False)}


@pytest.fixture(scope="module")
def chain(golden_dir):
    g = dict(np.load(f"{golden_dir}/gate_chain.npz"))
    n, places, seed, k = (int(x) for x in g["params"])
    plan = tuple((int(f), float(p)) for f, p in g["plan"])
    g["seq"] = synthetic.make_sequence(n, places, seed, plan)
    g["imu"] = synthetic.imu_log(g["seq"])
    g["k"], (g["thr"], g["gap"]) = k, (float(x) for x in g["thr_gap"])
    g["counts"] = json.loads(str(g["counts"]))
    return g


def test_fixture_floor_labels(chain):
    lab = opipe.floor_labels(chain["seq"].t, chain["imu"])
    assert np.array_equal(lab, chain["labels"])
    prod, events = floor_labels_from_imu(chain["seq"].t, chain["imu"])
    assert np.array_equal(prod, chain["labels"]) and len(events) == len(chain["seq"].rides)


@pytest.mark.parametrize("cfg", list(CFG))
def test_fixture_chain_reproduces(chain, cfg):
    verdict = {tuple(p): {"is_valid": bool(v)} for p, v in zip(chain["pairs"].tolist(), chain["pair_valid"])}
    rg, vg = CFG[cfg]
    r = opipe.gate_chain(chain["labels"], chain["desc"], chain["seq"].t, None, lambda a, b: verdict[(a, b)],
                         chain["gap"], chain["thr"], chain["k"], retrieval_gating=rg, verifier_gating=vg)
    for key in ("q", "m", "valid", "skip", "geo_valid", "gate_valid"):
        assert np.array_equal(r[key], chain[f"{cfg}_{key}"]), key
    assert r["counts"] == chain["counts"][cfg]


def test_fixture_one_pair_end_to_end(chain):
    """One fixture pair recomputed from pixels by the fp32 oracle (SuperPoint, LightGlue,
    OpenCV's RANSAC loop, decision rule)."""
    from mlgate.weights import lightglue_state_dict, superpoint_state_dict
    i = int(np.flatnonzero(chain["pair_valid"])[0])
    a, b = (int(x) for x in chain["pairs"][i])
    fr = synthetic.frames_host(chain["seq"], [a, b])
    r = opipe.verify_pair(fr[0], fr[1], superpoint_state_dict(0), opipe.make_matcher(lightglue_state_dict(0)),
                          ogeo.ISEC_K)
    assert r["is_valid"] and r["num_matches"] == chain["pair_matches"][i]
    assert r["num_inliers"] == chain["pair_inliers"][i]


def test_synthetic_sequence_shapes():
    seq = synthetic.make_sequence(40, 8, 3)
    a = synthetic.frames_host(seq, [0, 5])
    b = synthetic.frames_host(seq, [0, 5])
    assert a.shape == (2, 480, 640, 3) and a.dtype == np.uint8 and np.array_equal(a, b)
    assert set(np.unique(seq.shift)) <= {-8, 0, 8}
    assert np.all(seq.floor_gt[seq.place_of < 0] == 0)


def test_cv_rng_and_update_rule():
    r = ogeo.CvRng()
    s = [r.next() for _ in range(3)]
    # state' = (uint32)state * 4164903690 + (state >> 32) from state = 2^64 - 1
    st = (1 << 64) - 1
    for v in s:
        st = ((st & 0xFFFFFFFF) * 4164903690 + (st >> 32)) & ((1 << 64) - 1)
        assert v == st & 0xFFFFFFFF
    assert ogeo.update_num_iters(0.999, 0.5, 5, 1000) == int(np.rint(np.log(0.001) / np.log(1 - 0.5 ** 5)))
    assert ogeo.update_num_iters(0.999, 0.99, 5, 1000) == 1000  # budget never grows
    assert ogeo.update_num_iters(0.999, 0.0, 5, 1000) == 0  # all inliers: the loop ends


def test_cv_ransac_recovers_synthetic_geometry():
    rng = np.random.default_rng(4)
    k1, k2, R, t, inl = ogeo.synthetic_pair(rng, 200, 60, 0.5)
    E, mask, n_in = ogeo.cv_ransac(k1, k2, ogeo.ISEC_K, 3.0)
    assert n_in == int(mask.sum()) and np.sum(mask & inl) >= 0.95 * inl.sum() and np.sum(mask & ~inl) <= 5


def test_floor_codes_follow_python_equality():
    codes, has = floor_codes([1, 1.0, 2, None, float('nan'), float('nan'), np.int64(2), 'x', 'x'])
    assert codes[0] == codes[1] and codes[2] == codes[6] and codes[7] == codes[8]
    assert codes[4] != codes[5] and has.tolist() == [1, 1, 1, 0, 1, 1, 1, 1, 1]


def test_gate_nan_label_accepted_like_reference():
    g = SemanticLoopClosureGate(np.array([1.0, np.nan, 1.0]))
    assert g.gate_candidate(0, 1).is_valid  # abs(nan) > 0 is False in the reference
    v, rj = SemanticLoopClosureGate(np.array([1.0, np.nan, 1.0])).gate_candidates([(0, 1, 0.5), (0, 2, 0.4)])
    assert len(v) == 2 and not rj


def test_large_k_has_no_limit_and_k0_needs_no_device():
    """k has no upper limit (the reference's argsort()[:k]; k > 4096 runs the windowed
    radix select, tests/test_retrieval_gpu.py::test_k_beyond_4096_windows): a large k
    reaches the device (here: the no-device error, not a ValueError); k <= 0 returns the
    reference's empty list before any device work."""
    from mlgate._native import MlgateError
    spr = SemanticPlaceRecognition('cricavpr', device='cuda')
    spr.vpr.descriptors = [PlaceDescriptor(timestamp=float(i), descriptor=np.ones(4, np.float32), floor_label=1)
                           for i in range(4097)]
    assert spr.find_loop_closures(k=0) == []
    with pytest.raises(MlgateError):
        spr.find_loop_closures(k=5000)


def test_decision_fixture_one_pair_fp32(golden_dir):
    """tests/golden/decision_sample.npz (tools/decision_sample.py on the GPU +
    tools/decision_check_cpu.py here): its fp32 columns are the oracle chain's -- one
    valid sampled pair recomputed from pixels -- and the GPU decisions flip none of them."""
    import bench
    from mlgate.weights import lightglue_state_dict, superpoint_state_dict
    d = np.load(f"{golden_dir}/decision_sample.npz")
    assert len(d["a"]) == 600 and int(np.sum(d["is_valid"] != d["fp32_is_valid"])) == 0
    i = int(np.flatnonzero(d["fp32_is_valid"])[0])
    seq, _ = bench.sequence(int(d["keyframes"]), int(d["places"]))
    fr = synthetic.frames_host(seq, [int(d["a"][i]), int(d["b"][i])])
    r = opipe.verify_pair(fr[0], fr[1], superpoint_state_dict(0), opipe.make_matcher(lightglue_state_dict(0)),
                          ogeo.ISEC_K)
    assert r["is_valid"] and r["num_matches"] == d["fp32_matches"][i] and r["num_inliers"] == d["fp32_inliers"][i]
