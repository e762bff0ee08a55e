"""The drop-in API on the GPU, exercised the way the reference's demo and README use it
(place_recognition.py:994-1039, README.md:180-202), checked against golden vectors
captured from the reference and against the CPU oracle."""
import glob
import json
import os
import warnings

import numpy as np
import pytest
import torch

import mlgate
from mlgate.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
SIM_TOL = 4e-6  # see test_retrieval_gpu.py


def load(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "knn_*.npz"))), ids=os.path.basename)
def test_find_loop_closures_drop_in(dev, path):
    g = dict(np.load(path, allow_pickle=False))
    k, thr, gap, gating = g["params"]
    spr = mlgate.SemanticPlaceRecognition("mixvpr", device="cuda", similarity_threshold=float(thr),
                                          min_time_gap=float(gap))
    X = g["desc"].astype(np.float32)
    for i in range(len(X)):  # the reference's own demo injects descriptors this way (:1020)
        spr.vpr.descriptors.append(mlgate.PlaceDescriptor(
            timestamp=float(g["t"][i]), descriptor=X[i],
            floor_label=int(g["floor"][i]) if g["has_floor"][i] else None))
    ms = spr.find_loop_closures(enable_floor_gating=bool(gating), k=int(k))
    assert [m.query_idx for m in ms] == g["q"].tolist()
    assert [m.match_idx for m in ms] == g["m"].tolist()
    assert [m.is_valid for m in ms] == g["valid"].astype(bool).tolist()
    assert [m.query_timestamp for m in ms] == g["qt"].tolist()
    assert [m.match_timestamp for m in ms] == g["mt"].tolist()
    assert all(isinstance(m.similarity, float) for m in ms)
    assert np.max(np.abs(np.array([m.similarity for m in ms]) - g["sim"]), initial=0) <= SIM_TOL
    st, ref = spr.get_statistics(ms), json.loads(str(g["stats"]))
    assert set(st) == set(ref)
    for key in ("total_matches", "valid_matches", "rejected_matches", "rejection_rate"):
        assert st[key] == ref[key]
    for key in set(ref) - {"total_matches", "valid_matches", "rejected_matches", "rejection_rate"}:
        assert abs(st[key] - ref[key]) <= SIM_TOL


def test_single_descriptor_returns_empty(dev):
    spr = mlgate.SemanticPlaceRecognition("cricavpr", device="cuda")
    spr.vpr.descriptors.append(mlgate.PlaceDescriptor(0.0, np.ones(768, np.float32), floor_label=1))
    assert spr.find_loop_closures() == []


def test_pairwise_and_matrix_drop_in(dev):
    g = load("pairwise.npz")
    vpr = mlgate.CricaVPR(device="cuda")
    X = g["desc"].astype(np.float32)
    for i in range(len(X)):
        vpr.descriptors.append(mlgate.PlaceDescriptor(timestamp=float(i), descriptor=X[i]))
    assert np.array_equal(vpr.build_descriptor_matrix(), g["M"])
    S = vpr.compute_all_pairwise_similarities()
    assert S.dtype == np.float32 and np.max(np.abs(S - g["S"])) <= SIM_TOL


def test_query_drop_in(dev):
    g = load("query.npz")
    vpr = mlgate.MixVPR(device="cuda")
    vpr.extract_descriptor = lambda image: g["qdesc"].astype(np.float32)
    X = g["desc"].astype(np.float32)
    for i in range(len(X)):
        vpr.descriptors.append(mlgate.PlaceDescriptor(timestamp=float(g["t"][i]), descriptor=X[i]))
    for tag, ts, k, gap in (("a", 20.0, 5, 10.0), ("b", None, 5, 10.0), ("c", 100.0, 12, 30.0)):
        ms = vpr.query(None, timestamp=ts, k=k, min_time_gap=gap)
        assert [m.match_idx for m in ms] == g[f"{tag}_m"].tolist()
        assert [m.query_idx for m in ms] == g[f"{tag}_q"].tolist()
        assert np.max(np.abs(np.array([m.similarity for m in ms]) - g[f"{tag}_sim"]), initial=0) <= SIM_TOL
    sims = vpr._compute_similarity(g["qdesc"], X)
    ref = (X / (np.linalg.norm(X, axis=1, keepdims=True) + 1e-8)) @ (g["qdesc"] / (np.linalg.norm(g["qdesc"]) + 1e-8))
    assert np.max(np.abs(sims - ref)) <= SIM_TOL


def test_cross_correlation_and_rerank_drop_in(dev):
    g = load("xcorr.npz")
    feats = g["feats"].astype(np.float32)
    vpr = mlgate.CricaVPR(device="cuda", use_reranking=True)
    for (a, b), ref in zip(g["pairs"], g["scores"]):
        assert abs(vpr.compute_cross_correlation_score(feats[a], feats[b]) - ref) < 1e-5
    assert abs(vpr.compute_cross_correlation_score(feats[0][0], feats[1][0]) - float(g["s2d"])) < 1e-5
    for i in range(5):
        vpr._feature_cache[i] = feats[i]
    cands = [(int(j), float(s)) for j, s in g["cands"]]
    rr = vpr.rerank_candidates(0, cands, top_k=4)
    assert [j for j, _ in rr] == [int(j) for j in g["rr"][:, 0]]
    assert np.allclose([s for _, s in rr], g["rr"][:, 1], rtol=0, atol=1e-5)
    assert vpr.rerank_candidates(5, cands, top_k=3) == [tuple(x) for x in cands[:3]]


def _scene(rng):
    img = np.zeros((480, 640, 3), np.uint8)
    for _ in range(25):
        x, y = rng.integers(0, 580), rng.integers(0, 420)
        img[y:y + rng.integers(20, 120), x:x + rng.integers(20, 120)] = rng.integers(60, 255, 3)
    return np.clip(img.astype(np.int32) + rng.integers(0, 30, img.shape), 0, 255).astype(np.uint8)


def test_cricavpr_add_image_end_to_end(dev):
    from oracle import vit as ovit
    rng = np.random.default_rng(7)
    imgs = [_scene(rng) for _ in range(3)]
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        spr = mlgate.SemanticPlaceRecognition("cricavpr", device="cuda")
        d0 = spr.add_image(imgs[0], 0.0, 5)
    assert any("synthetic" in str(x.message) for x in w)
    spr.add_images(imgs[1:], [20.0, 40.0], [5, 1])
    osd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(0).items()}
    for i, im in enumerate(imgs):
        ref = ovit.extract_descriptor(im, osd)
        got = spr.vpr.descriptors[i].descriptor
        assert got.dtype == np.float32 and got.shape == (768,)
        cos = float(np.dot(got, ref) / np.linalg.norm(got) / np.linalg.norm(ref))
        assert 1 - cos < 1e-4
        assert tuple(spr.vpr._feature_cache[i].shape) == (1, 528, 768)
    assert d0 is spr.vpr.descriptors[0] and d0.floor_label == 5
    single = spr.vpr.extract_descriptor(imgs[0])
    assert np.allclose(single, spr.vpr.descriptors[0].descriptor, rtol=0, atol=1e-6)
    lf = spr.vpr.extract_local_features(imgs[0])
    assert lf.shape == (1, 528, 768) and lf.dtype == np.float32
    ms = spr.find_loop_closures(k=2)
    assert all(m.query_idx != m.match_idx for m in ms)


def test_anyloc_end_to_end(dev):
    from oracle import vit as ovit
    rng = np.random.default_rng(8)
    img = _scene(rng)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        vpr = mlgate.AnyLoc(device="cuda")
        got = vpr.extract_descriptor(img)
    ref = ovit.anyloc_descriptor(img, {k: torch.from_numpy(v) for k, v in synthetic_state_dict(0).items()})
    cos = float(np.dot(got, ref) / np.linalg.norm(got) / np.linalg.norm(ref))
    assert got.shape == (768,) and 1 - cos < 1e-4


def test_resnet_methods_refuse_cpu_device(dev):
    """The ResNet-50 fallback runs on the GPU only: device='cpu' raises, never a CPU path."""
    with pytest.raises(mlgate._native.MlgateError):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            mlgate.MixVPR(device="cpu").extract_descriptor(np.zeros((480, 640, 3), np.uint8))
