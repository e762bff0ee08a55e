"""The image-level drop-in verification API on the GPU (geometric_verification.py:196-744)
against the fp32 oracle chain's per-pair verdicts (tests/golden/gate_chain.npz: SuperPoint
+ LightGlue in fp32 and OpenCV's RANSAC loop on the seeded 40-keyframe sequence).

Covers the paths the batched gate does not call: LightGlue.detect_and_match on numpy
images, GeometricVerifier.verify / verify_batch, the verify branch of
SemanticGeometricVerifier.verify_with_semantics, and the SuperGlue matcher's fallback
(the reference resolves it to LightGlue; LoFTR is native: tests/test_loftr_gpu.py).

Bar: is_valid identical to the fp32 chain on every pair; number of matches within 10 %
and inliers within 15 % of the fp32 chain (bf16 GEMMs move a few percent of matches);
the batched and per-pair APIs give identical results.
"""
import warnings

import numpy as np
import pytest

from mlgate import synthetic
from mlgate.verify import GeometricVerifier, LightGlue, SemanticGeometricVerifier
from oracle import geometry as ogeo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def chain(golden_dir):
    g = dict(np.load(f"{golden_dir}/gate_chain.npz"))
    n, places, seed, _ = (int(x) for x in g["params"])
    plan = tuple((int(f), float(p)) for f, p in g["plan"])
    g["frames"] = synthetic.frames_host(synthetic.make_sequence(n, places, seed, plan))
    valid = np.flatnonzero(g["pair_valid"])[:3]
    invalid = np.flatnonzero(~g["pair_valid"].astype(bool) & (g["pair_matches"] >= 5))[:3]
    g["sel"] = np.r_[valid, invalid]
    return g


def _images(chain, i):
    a, b = chain["pairs"][i]
    return chain["frames"][a], chain["frames"][b]


def _check(chain, i, r):
    assert r.is_valid == bool(chain["pair_valid"][i]), (i, r)
    ref_m, ref_in = int(chain["pair_matches"][i]), int(chain["pair_inliers"][i])
    assert abs(r.num_matches - ref_m) <= max(3, 0.10 * ref_m), (i, r.num_matches, ref_m)
    if r.is_valid:
        assert abs(r.num_inliers - ref_in) <= 0.15 * ref_in, (i, r.num_inliers, ref_in)
        assert r.relative_pose is not None and r.relative_pose.shape == (4, 4)


def test_detect_and_match_on_images(dev, chain):
    lg = LightGlue(device=str(dev))
    for i in chain["sel"]:
        k1, k2, sc = lg.detect_and_match(*_images(chain, i))
        assert k1.dtype == np.float32 and k1.shape == k2.shape and k1.shape == (len(sc), 2)
        ref = int(chain["pair_matches"][i])
        assert abs(len(k1) - ref) <= max(3, 0.10 * ref), (i, len(k1), ref)
        assert np.all((sc > 0) & (sc <= 1))


def test_verify_and_verify_batch(dev, chain):
    v = GeometricVerifier('lightglue', device=str(dev))
    single = [v.verify(*_images(chain, i), K=ogeo.ISEC_K, query_idx=int(i), match_idx=int(i) + 1)
              for i in chain["sel"]]
    for i, r in zip(chain["sel"], single):
        assert (r.query_idx, r.match_idx) == (int(i), int(i) + 1)
        _check(chain, i, r)
    batch = v.verify_batch([_images(chain, i) for i in chain["sel"]], K=ogeo.ISEC_K,
                           indices=[(int(i), int(i) + 1) for i in chain["sel"]])
    for a, b in zip(single, batch):
        assert (a.query_idx, a.match_idx, a.num_matches, a.num_inliers, a.is_valid) == \
            (b.query_idx, b.match_idx, b.num_matches, b.num_inliers, b.is_valid)
        assert a.inlier_ratio == b.inlier_ratio


def test_verify_without_K_uses_fundamental(dev, chain):
    v = GeometricVerifier('lightglue', device=str(dev))
    i = chain["sel"][0]
    r = v.verify(*_images(chain, i), K=None)
    assert r.relative_pose is None and r.essential_matrix is not None and r.essential_matrix.shape == (3, 3)
    assert r.num_matches > 0


def test_verify_with_semantics_verify_branch(dev, chain):
    v = SemanticGeometricVerifier('lightglue', device=str(dev))
    labels = chain["labels"]
    for i in chain["sel"]:
        a, b = chain["pairs"][i]
        r = v.verify_with_semantics(*_images(chain, i), int(labels[a]), int(labels[a]), K=ogeo.ISEC_K,
                                    query_idx=int(a), match_idx=int(b))
        _check(chain, i, r)
    r = v.verify_with_semantics(*_images(chain, chain["sel"][0]), 1, 2, K=ogeo.ISEC_K)
    assert not r.is_valid and r.num_matches == 0
    st = v.get_statistics()
    nv = int(chain["pair_valid"][chain["sel"]].sum())
    assert st["verified"] == len(chain["sel"]) and st["skipped_floor_mismatch"] == 1
    assert st["valid"] == nv and st["invalid"] == len(chain["sel"]) - nv
    assert st["total_candidates"] == len(chain["sel"]) + 1


@pytest.mark.parametrize("name,msg", [("superglue", "SuperGlue not installed")])
def test_fallback_matchers_equal_lightglue(dev, chain, name, msg):
    base = GeometricVerifier('lightglue', device=str(dev))
    v = GeometricVerifier(name, device=str(dev))
    pairs = [_images(chain, i) for i in chain["sel"][:2]]
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        got = [v.verify(a, b, K=ogeo.ISEC_K) for a, b in pairs]
    assert any(msg in str(x.message) for x in w)
    want = [base.verify(a, b, K=ogeo.ISEC_K) for a, b in pairs]
    for a, b in zip(got, want):
        assert (a.num_matches, a.num_inliers, a.is_valid) == (b.num_matches, b.num_inliers, b.is_valid)
