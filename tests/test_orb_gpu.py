"""ORB + BFMatcher fallback on the GPU (csrc/orb.hip) against the CPU oracle
(oracle/csrc/orb.c), bit for bit: keypoints, levels, Harris responses, angles,
descriptors, cross-checked matches and their order, and the drop-in
LightGlue._detect_and_match_fallback (geometric_verification.py:314-350) selected by
MLGATE_LIGHTGLUE_FALLBACK=orb.  Parity with OpenCV itself is unpinned (see
oracle/csrc/orb.c)."""
import warnings

import numpy as np
import pytest
import torch

from mlgate import synthetic
from mlgate.orb import OrbGPU
from oracle import orb as oorb

pytestmark = pytest.mark.gpu


def _frame(seed, H=480, W=640, shift=(0, 0), noise=20):
    rng = np.random.default_rng(seed)
    base = synthetic.scene(seed % 7, H, W)
    img = np.roll(base, shift[::-1], (0, 1)).astype(int) + rng.integers(0, noise, base.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


@pytest.fixture(scope="module")
def orb_gpu(dev):
    return OrbGPU(device="cuda", nfeatures=2048)


@pytest.mark.parametrize("H,W", [(480, 640), (540, 720), (120, 160)])
def test_detect_matches_oracle(orb_gpu, H, W):
    frames = np.stack([_frame(s, H, W) for s in range(3)])
    kp, resp, ang, lev, desc, cnt = orb_gpu.detect_device(torch.from_numpy(frames).cuda())
    kp, resp, ang, lev, desc, cnt = (t.cpu().numpy() for t in (kp, resp, ang, lev, desc, cnt))
    for f in range(len(frames)):
        rk, rl, rr, ra, rd = oorb.detect_and_compute(oorb.gray(frames[f]), 2048)
        n = cnt[f]
        assert n == len(rk) and n > 0
        assert np.array_equal(kp[f, :n], rk)
        assert np.array_equal(lev[f, :n], rl)
        assert np.array_equal(resp[f, :n], rr)
        assert np.array_equal(ang[f, :n], ra)
        assert np.array_equal(desc[f, :n], rd)


def test_match_matches_oracle(orb_gpu):
    frames = np.stack([_frame(1), _frame(1, shift=(8, -8)), _frame(2), _frame(1, shift=(-16, 0))])
    kp, _, _, _, desc, cnt = orb_gpu.detect_device(torch.from_numpy(frames).cuda())
    pairs = [(0, 1), (0, 2), (3, 0), (1, 3)]
    q, t, d, n = orb_gpu.match_device(desc, cnt, [a for a, _ in pairs], [b for _, b in pairs])
    q, t, d, n = q.cpu().numpy(), t.cpu().numpy(), d.cpu().numpy(), n.cpu().numpy()
    dh, ch = desc.cpu().numpy(), cnt.cpu().numpy()
    for p, (a, b) in enumerate(pairs):
        rq, rt, rd = oorb.bf_match(dh[a, :ch[a]], dh[b, :ch[b]])
        m = n[p]
        assert m == len(rq)
        assert np.array_equal(q[p, :m], rq) and np.array_equal(t[p, :m], rt) and np.array_equal(d[p, :m], rd)
    assert n[0] > 50  # a revisit (8-px shift) matches


def test_dropin_fallback_equals_oracle(dev, monkeypatch):
    import mlgate
    monkeypatch.setenv("MLGATE_LIGHTGLUE_FALLBACK", "orb")
    a, b = _frame(3), _frame(3, shift=(8, 8))
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        lg = mlgate.LightGlue(device="cuda")
        m1, m2, conf = lg.detect_and_match(a, b)
    assert any("ORB+BFMatcher fallback" in str(x.message) for x in w)
    assert lg._is_native is False
    r1, r2, rc = oorb.detect_and_match_fallback(a, b)
    assert m1.dtype == r1.dtype and np.array_equal(m1, r1) and np.array_equal(m2, r2) and np.array_equal(conf, rc)
    good = np.abs((m2 - m1) - 8).max(1) < 1.5
    assert good.mean() > 0.5
    # the verifier on top of it (geometric_verification.py:564-620)
    v = mlgate.GeometricVerifier(matcher_type='lightglue', device='cuda')
    res = v.verify(a, b)
    assert res.num_matches == len(r1)
    # batched device path == per pair
    frames = torch.from_numpy(np.stack([a, b, _frame(4)])).cuda()
    out = lg.detect_and_match_batch(frames, [(0, 1), (2, 0)])
    assert np.array_equal(out[0][0], r1) and np.array_equal(out[0][2], rc)
    s1, s2, sc = oorb.detect_and_match_fallback(_frame(4), a)
    assert np.array_equal(out[1][0], s1) and np.array_equal(out[1][1], s2) and np.array_equal(out[1][2], sc)


def test_dropin_fallback_identical_frames_raise_like_reference(dev, monkeypatch):
    import mlgate
    monkeypatch.setenv("MLGATE_LIGHTGLUE_FALLBACK", "orb")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        lg = mlgate.LightGlue(device="cuda")
        img = synthetic.scene(2)
        with pytest.raises(ZeroDivisionError):
            lg.detect_and_match(img, img.copy())
        flat = np.full((480, 640, 3), 128, np.uint8)  # no corners -> the reference's empty result
        m1, m2, c = lg.detect_and_match(flat, img)
    assert len(m1) == 0 and len(m2) == 0 and len(c) == 0
