"""CPU checks of the RANSAC / pose oracle (oracle/geometry.py) on exact synthetic
geometry: the minimal solvers recover the true model, the errors vanish on exact
correspondences, and recoverPose returns the true (R, t)."""
import numpy as np
import pytest

from oracle import geometry as G


def _exact(seed, n):
    rng = np.random.default_rng(seed)
    k1, k2, R, t, inl = G.synthetic_pair(rng, n, 0, noise_px=0.0)
    return k1.astype(np.float64), k2.astype(np.float64), R, t


def _close_up_to_sign(A, B, tol):
    A = A / np.linalg.norm(A)
    B = B / np.linalg.norm(B)
    return min(np.abs(A - B).max(), np.abs(A + B).max()) < tol


@pytest.mark.parametrize("seed", range(5))
def test_five_point_recovers_true_essential(seed):
    k1, k2, R, t = _exact(seed, 5)
    Es = G.five_point(G.normalize(k1, G.ISEC_K), G.normalize(k2, G.ISEC_K))
    Et = G.essential_from_pose(R, t)
    assert 1 <= len(Es) <= 10
    assert any(_close_up_to_sign(E, Et, 1e-5) for E in Es)


@pytest.mark.parametrize("seed", range(5))
def test_seven_point_recovers_true_fundamental(seed):
    k1, k2, R, t = _exact(100 + seed, 7)
    Fs = G.seven_point(k1, k2)
    Ft = G.fundamental_from_pose(R, t, G.ISEC_K)
    assert 1 <= len(Fs) <= 3
    assert any(_close_up_to_sign(F, Ft, 1e-4) for F in Fs)


def test_errors_vanish_on_exact_correspondences():
    k1, k2, R, t = _exact(7, 200)
    Et = G.essential_from_pose(R, t)
    e = G.sampson_error(Et, G.normalize(k1, G.ISEC_K), G.normalize(k2, G.ISEC_K))
    assert e.max() < 1e-13  # float32-rounded pixels
    f = G.epiline_error(G.fundamental_from_pose(R, t, G.ISEC_K), k1, k2)
    assert f.max() < 1e-6


@pytest.mark.parametrize("seed", range(4))
def test_recover_pose_returns_truth(seed):
    k1, k2, R, t = _exact(200 + seed, 60)
    good, Rr, tr = G.recover_pose(G.essential_from_pose(R, t), k1, k2, G.ISEC_K)
    assert good == 60
    assert G.rotation_angle_deg(Rr, R) < 1e-6
    assert np.allclose(tr, t, atol=1e-6)


# --- the compiled twin (oracle/csrc/ransac_cv.c) against the numpy restatement --------
@pytest.mark.parametrize("seed", range(6))
def test_c_five_point_equals_numpy_five_point(seed):
    from oracle import _lib
    rng = np.random.default_rng(100 + seed)
    k1, k2, _, _, _ = G.synthetic_pair(rng, 5, 0, noise_px=0.3)
    p1, p2 = G.normalize(k1, G.ISEC_K), G.normalize(k2, G.ISEC_K)
    A, B = G.five_point(p1, p2), _lib.five_point(p1, p2)
    assert len(A) == len(B)
    for E in A:
        assert any(_close_up_to_sign(E, F, 1e-7) for F in B)


@pytest.mark.parametrize("seed", range(8))
def test_c_essential_ransac_equals_numpy_restatement(seed):
    """Same sample stream, same acceptance rule: identical inlier counts and masks."""
    from oracle import _lib
    rng = np.random.default_rng(200 + seed)
    n_in = int(rng.integers(30, 250))
    k1, k2, _, _, _ = G.synthetic_pair(rng, n_in, int(rng.integers(0, n_in // 2 + 1)), noise_px=0.8)
    _, mask_py, g_py = G.cv_ransac(k1, k2, G.ISEC_K, 3.0)
    _, mask_c, g_c = _lib.essential_ransac(k1, k2, G.ISEC_K, 3.0)
    assert g_c == g_py
    assert np.array_equal(mask_c, mask_py)


def test_c_essential_ransac_degenerate_sizes():
    from oracle import _lib
    rng = np.random.default_rng(7)
    k1, k2, _, _, _ = G.synthetic_pair(rng, 5, 0, noise_px=0.0)
    assert _lib.essential_ransac(k1[:4], k2[:4], G.ISEC_K)[2] == 0
    _, mask, g = _lib.essential_ransac(k1, k2, G.ISEC_K)
    assert g == 5 and mask.all()


# --- rs_math.h (shared by the GPU RANSAC and the C twin) against the library maths -----
def test_rs_math_helpers_track_libm():
    """rs_log / rs_root replace libm inside both RANSACs (so the two agree bit for bit);
    they must still be the functions they stand for: log within 2 ulp, the Aberth start
    radius within 4e-15, and RANSACUpdateNumIters identical to the numpy restatement
    (np.log, **) on a sweep of inlier ratios and budgets."""
    from oracle import _lib
    L = _lib.lib()
    rng = np.random.default_rng(3)
    xs = np.concatenate([np.exp(rng.uniform(-700, 700, 4000)), rng.uniform(0.5, 2.0, 4000), [1.0, 0.001, 1e-300]])
    for x in xs:
        got, want = L.orc_rs_log(float(x)), float(np.log(x))
        assert abs(got - want) <= 2 * np.spacing(abs(want)) + 1e-300, (x, got, want)
    for x in np.exp(rng.uniform(-60, 60, 2000)):
        for n in range(1, 11):
            got, want = L.orc_rs_root(float(x), n), float(x) ** (1.0 / n)
            assert abs(got - want) <= 4e-15 * want, (x, n, got, want)
    assert L.orc_rs_root(0.0, 4) == 0.0
    for m in (5, 7):
        for n in (20, 100, 1000, 2048):
            for g in range(m, n + 1, max(1, n // 300)):
                ep = (n - g) / n
                for budget in (1000, 400, 37):
                    assert L.orc_rs_update_iters(0.999, ep, m, budget) == G.update_num_iters(0.999, ep, m, budget), \
                        (m, n, g, budget)


@pytest.mark.parametrize("seed", range(6))
def test_c_fundamental_ransac_equals_numpy_restatement(seed):
    """>= 15 matches without K: the same sample stream (with the collinearity redraw) and
    acceptance rule.  The twin solves on Hartley-normalised points as the GPU does, numpy
    on pixels as OpenCV's run7Point; the inlier counts agree (a point within rounding of
    the threshold may flip: <= 0.5 %)."""
    from oracle import _lib
    rng = np.random.default_rng(300 + seed)
    n_in = int(rng.integers(40, 300))
    k1, k2, _, _, _ = G.synthetic_pair(rng, n_in, int(rng.integers(0, n_in // 3 + 1)), noise_px=0.5)
    _, mask_py, g_py = G.cv_ransac(k1, k2, None, 3.0)
    F, mask_c, g_c = _lib.fundamental_ransac(k1, k2, 3.0)
    assert abs(g_c - g_py) <= max(1, 0.005 * len(k1)), (g_c, g_py)
    assert np.array_equal(mask_c, G.inlier_mask(F, k1, k2, None, 3.0))


def test_c_fundamental_small_sizes():
    from oracle import _lib
    rng = np.random.default_rng(8)
    k1, k2, _, _, _ = G.synthetic_pair(rng, 12, 0, noise_px=0.2)
    assert _lib.fundamental_ransac(k1[:6], k2[:6])[2] == 0
    F, mask, g = _lib.fundamental_ransac(k1[:7], k2[:7])
    assert g == 7 and mask.all() and F is not None
    F, mask, g = _lib.fundamental_ransac(k1, k2)  # LMedS: mask = the sigma test of the model
    e = G.epiline_error(F, k1, k2)
    med = np.sort(e)[len(e) // 2]
    sigma = max(2.5 * 1.4826 * (1 + 5.0 / (len(e) - 7)) * np.sqrt(np.float64(med)), 0.001)
    assert np.array_equal(mask, e <= np.float32(sigma * sigma)) and g == int(mask.sum())


def test_bench_fixture_records_ransac_twin_equality():
    """The committed bench-scale fixture (tools/bench_parity.py chain on the GPU box, round 6)
    records the GPU RANSAC against the C twin on every ordered pair of a bench step, on the
    product's match lists and on the fp32 chain's: counts, masks and (fixtures made since the
    model check was added) the model bits equal on all of them."""
    import json
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "bench_chain_fp32.npz"))
    rep = json.loads(str(z["report"]))
    for key in ("twin_product", "twin_fp32"):
        r = rep[key]
        assert r["pairs"] > 32000 and r["inliers_equal_c_twin"] == 1.0 and r["masks_equal_c_twin"] == 1.0, r
        assert r.get("models_equal_c_twin", 1.0) == 1.0, r
