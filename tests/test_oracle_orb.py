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
        assert np.array_equal(sc[:8], scales) and np.array_equal(sc[8:], oorb.gauss_kernel())
        assert ip[24:40].tolist() == oorb.umax_table()[:16].tolist()
        assert ip[40:].tolist() == [20, 31]
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
    k = oorb.gauss_kernel().astype(np.float64)
    assert abs(k.sum() - 1) < 1e-6 and np.array_equal(k, k[::-1]) and k.argmax() == 3


def test_gauss_kernel_is_opencv_bitexact_kernel():
    """getGaussianKernelBitExact(7, 2) in float64 rounded to float32; the taps are the
    sigma-2 Gaussian normalised to sum 1 (the old per-tap float path agrees to 1 ulp)."""
    x = np.arange(7) - 3.0
    g = np.exp(-x * x / 8.0)
    k = oorb.gauss_kernel()
    assert k.dtype == np.float32
    assert np.allclose(k, g / g.sum(), rtol=2e-7, atol=0)
    assert k[3] == np.float32(1.0 / (2 * g[:3].sum() + 1.0))


def _resize_exact_py(src, DH, DW):
    """INTER_LINEAR_EXACT on 8U restated with Python ints / floats (resize_bitExact)."""
    H, W = src.shape

    def axis(d, dsize, ssize):
        scale = 1.0 / (dsize / ssize)
        f = scale * (d + 0.5) - 0.5
        i = int(np.floor(f))
        if i < 0 or ssize <= 1:
            return 0, 0
        if i >= ssize - 1:
            return ssize - 1, 0
        return i, int(round((f - i) * 256.0))  # Python round: half to even, as cvRound

    out = np.zeros((DH, DW), np.uint8)
    for y in range(DH):
        y0, cy1 = axis(y, DH, H)
        y1 = min(y0 + 1, H - 1)
        for x in range(DW):
            x0, cx1 = axis(x, DW, W)
            x1 = min(x0 + 1, W - 1)
            h0 = (256 - cx1) * int(src[y0, x0]) + cx1 * int(src[y0, x1])
            h1 = (256 - cx1) * int(src[y1, x0]) + cx1 * int(src[y1, x1])
            out[y, x] = (h0 * (256 - cy1) + h1 * cy1 + 32768) >> 16
    return out


def _blur_py(img, k):
    """sepFilter2D(8U, float kernel) with REFLECT_101 restated in numpy float32."""
    H, W = img.shape
    k = k.astype(np.float32)
    xs = np.abs(np.arange(-3, W + 3))
    xs = np.where(xs >= W, 2 * W - 2 - xs, xs)
    src = img.astype(np.float32)
    h = k[0] * src[:, xs[0:W]]
    for t in range(1, 7):
        h = h + k[t] * src[:, xs[t:t + W]]
    ys = np.abs(np.arange(-3, H + 3))
    ys = np.where(ys >= H, 2 * H - 2 - ys, ys)
    s = k[3] * h
    for t in range(1, 4):
        s = s + k[3 + t] * (h[ys[3 + t:3 + t + H]] + h[ys[3 - t:3 - t + H]])
    return np.clip(np.rint(s), 0, 255).astype(np.uint8)


def test_pyramid_and_blur_restated_twice():
    """The C oracle's INTER_LINEAR_EXACT pyramid and float GaussianBlur equal the Python
    restatements above on a frame where every level and the borders are exercised."""
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, (61, 83), dtype=np.uint8)
    img[10:30, 20:50] = 200
    scales, ws, hs, _ = oorb.level_geometry(61, 83, 500)
    prev = img
    k = oorb.gauss_kernel()
    for l in range(1, 4):
        cur = _resize_exact_py(prev, int(hs[l]), int(ws[l]))
        assert np.array_equal(cur, oorb.resize_exact(prev, int(hs[l]), int(ws[l]))), l
        assert np.array_equal(_blur_py(cur, k), oorb.blur(cur)), l
        prev = cur
    # upscale edges clamp to the first / last pixel
    tiny = np.array([[0, 100], [200, 255]], np.uint8)
    assert np.array_equal(_resize_exact_py(tiny, 4, 4), oorb.resize_exact(tiny, 4, 4))


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
