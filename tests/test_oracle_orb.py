"""ORB + BFMatcher fallback (geometric_verification.py:244-248, 314-350): the CPU oracle
and the product's host-side geometry.  OpenCV is not installed, so parity with OpenCV
itself is UNPINNED; these tests pin the oracle's pieces against independent plain
restatements (FAST-9 segment test, Hamming brute force, the ORB_Impl level plan) and the
product geometry against the oracle's.  GPU-vs-oracle parity: tests/test_orb_gpu.py."""
import numpy as np
import pytest

from mlgate import orb as porb
from oracle import orb as oorb

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
          (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def test_level_plan_matches_opencv_defaults():
    scales, ws, hs, per = oorb.level_geometry(480, 640, 2048)
    assert ws.tolist() == [640, 533, 444, 370, 309, 257, 214, 179]
    assert hs.tolist() == [480, 400, 333, 278, 231, 193, 161, 134]
    assert per.sum() == 2048 and per[0] == 445 and per[-1] == 124
    assert np.allclose(scales, 1.2 ** np.arange(8), rtol=1e-6)
    # ISEC 720 x 540
    _, ws2, hs2, per2 = oorb.level_geometry(540, 720, 2048)
    assert ws2[1] == 600 and hs2[1] == 450 and per2.sum() == 2048


def test_product_geometry_equals_oracle():
    for H, W, n in ((480, 640, 2048), (540, 720, 2048), (97, 131, 500), (480, 640, 1000)):
        ip, sc = porb.geometry(H, W, n)
        scales, ws, hs, per = oorb.level_geometry(H, W, n)
        assert ip[:8].tolist() == ws.tolist() and ip[8:16].tolist() == hs.tolist()
        assert ip[16:24].tolist() == per.tolist()
        assert np.array_equal(sc, scales)
        assert ip[32:48].tolist() == oorb.umax_table()[:16].tolist()
        assert ip[48:55].tolist() == oorb.gauss_coeffs().tolist()
        assert ip[55:].tolist() == [20, 31]
    assert np.array_equal(porb.random_pattern().astype(np.int32), oorb.random_pattern())


def test_pattern_and_umax():
    pat = oorb.random_pattern()
    assert pat.shape == (512, 2) and pat.min() >= -15 and pat.max() <= 15
    # cv::RNG(0x34985739): first outputs of the multiply-with-carry stream
    s = 0x34985739
    s = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & ((1 << 64) - 1)
    assert pat[0, 0] == (s & 0xFFFFFFFF) % 31 - 15
    um = oorb.umax_table()
    assert um[0] == 15 and um[15] == 3 and (np.diff(um[:16]) <= 0).all()
    assert oorb.gauss_coeffs().sum() == 256


def _fast_slow(img, x, y, t):
    v = int(img[y, x])
    d = [int(img[y + dy, x + dx]) - v for dx, dy in CIRCLE]
    best = 0
    for tt in range(t, 256):  # largest tt at which 9 contiguous are all > v + tt or all < v - tt
        ok = any(all(d[(k + j) % 16] > tt for j in range(9)) or all(d[(k + j) % 16] < -tt for j in range(9))
                 for k in range(16))
        if not ok:
            break
        best = tt
    return best


def test_fast_scores_and_nms_against_segment_test():
    rng = np.random.default_rng(3)
    img = np.zeros((90, 100), np.uint8)
    for _ in range(25):
        x, y = rng.integers(0, 90), rng.integers(0, 70)
        img[y:y + rng.integers(5, 25), x:x + rng.integers(5, 25)] = rng.integers(40, 255)
    img = np.clip(img.astype(int) + rng.integers(0, 12, img.shape), 0, 255).astype(np.uint8)
    kp, lev, resp, ang, desc = oorb.detect_and_compute(img, 4000)
    l0 = kp[lev == 0].astype(int)
    assert len(l0) > 0
    # every level-0 keypoint is a FAST-9 corner at threshold 20 inside the 31-px border,
    # a strict 3x3 maximum of the score
    sc = np.zeros(img.shape, int)
    for y in range(3, img.shape[0] - 3):
        for x in range(3, img.shape[1] - 3):
            sc[y, x] = _fast_slow(img, x, y, 20) if _fast_slow(img, x, y, 20) > 20 or any(
                all((int(img[y + dy, x + dx]) - int(img[y, x])) * sg > 20 for dx, dy in
                    [CIRCLE[(k + j) % 16] for j in range(9)]) for k in range(16) for sg in (1, -1)) else 0
    want = set()
    for y in range(31, img.shape[0] - 31):
        for x in range(31, img.shape[1] - 31):
            s = sc[y, x]
            if s and all(sc[y + dy, x + dx] < s for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dx or dy):
                want.add((x, y))
    assert set(map(tuple, l0.tolist())) == want
    assert desc.shape == (len(kp), 32) and np.all((ang >= 0) & (ang < 360))


def test_bf_match_cross_check_against_bruteforce():
    rng = np.random.default_rng(5)
    d1 = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    d2 = np.concatenate([d1[:150] ^ (rng.random((150, 32)) < 0.03).astype(np.uint8),
                         rng.integers(0, 256, (120, 32), dtype=np.uint8)])
    q, t, dist = oorb.bf_match(d1, d2)
    D = np.unpackbits(d1[:, None, :] ^ d2[None, :, :], axis=2).sum(2)
    b12, b21 = D.argmin(1), D.argmin(0)  # first minimum, as BFMatcher
    keep = [i for i in range(len(d1)) if b21[b12[i]] == i]
    ref = sorted(((int(D[i, b12[i]]), i, int(b12[i])) for i in keep), key=lambda r: r[0])  # stable
    assert [(d, i, j) for d, i, j in zip(dist, q, t)] == ref
    assert len(ref) >= 140


def test_fallback_identical_frames_divides_by_zero():
    """All cross-checked distances 0 -> the reference's `1 - d / max_dist` raises."""
    from mlgate import synthetic
    with pytest.raises(ZeroDivisionError):
        oorb.detect_and_match_fallback(synthetic.scene(4), synthetic.scene(4))


@pytest.mark.parametrize("shift", [(8, -8), (-16, 8)])
def test_fallback_on_shifted_frames(shift):
    from mlgate import synthetic
    rng = np.random.default_rng(1)
    base = synthetic.scene(4)
    a = np.clip(base.astype(int) + rng.integers(0, 20, base.shape), 0, 255).astype(np.uint8)
    b = np.clip(np.roll(base, shift[::-1], (0, 1)).astype(int) + rng.integers(0, 20, base.shape), 0, 255)
    m1, m2, conf = oorb.detect_and_match_fallback(a, b.astype(np.uint8))
    assert len(m1) > 20
    good = np.abs((m2 - m1) - np.array(shift)).max(1) < 1.5
    assert good.mean() > 0.5
    assert conf.max() <= 1 and conf.min() >= 0 and np.all(np.diff(1 - conf) >= 0)
