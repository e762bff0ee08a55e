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
