"""Oracle for epipolar RANSAC and relative pose (test infrastructure only).

Restates, in numpy, the OpenCV calls of BaseFeatureMatcher
(scripts/semantic_gating/geometric_verification.py:104-188):
  * findEssentialMat(k1, k2, K, RANSAC, prob=0.999, threshold) -- points normalised
    by K, threshold / ((fx + fy) / 2), 5-point minimal solver, Sampson error
    (EMEstimatorCallback::computeError), inlier iff float32(err) <= float32(thr^2);
  * findFundamentalMat(k1, k2, FM_RANSAC, threshold, 0.999) -- 7-point solver,
    max of the two squared point-to-epiline distances (FMEstimatorCallback);
  * recoverPose(E, k1[in], k2[in], K) -- decomposeEssentialMat (SVD, det fixes,
    W = [[0,1,0],[-1,0,0],[0,0,1]]), DLT triangulation, cheirality with distance 50.
cv2 (an unpinned opencv-python) is not installed here and the reference has no tests
or fixtures for this path, so parity is unpinned beyond decisions: the GPU path is
checked against this restatement and against ground truth on seeded synthetic
geometry (known R, t, sub-pixel noise, far outliers), where any correct RANSAC
reaches the same inlier set and decision.
"""
import numpy as np

ISEC_K = np.array([[893.63, 0.0, 376.95], [0.0, 893.97, 266.57], [0.0, 0.0, 1.0]])


def normalize(k, K):
    k = np.asarray(k, np.float64)
    return np.stack([(k[:, 0] - K[0, 2]) / K[0, 0], (k[:, 1] - K[1, 2]) / K[1, 1]], 1)


def sampson_error(E, p1, p2):
    """float32 Sampson errors of normalised correspondences (cv2 EMEstimatorCallback)."""
    x1 = np.c_[p1, np.ones(len(p1))]
    x2 = np.c_[p2, np.ones(len(p2))]
    Ex1 = x1 @ E.T
    Etx2 = x2 @ E
    r = np.sum(x2 * Ex1, 1)
    return (r * r / (Ex1[:, 0] ** 2 + Ex1[:, 1] ** 2 + Etx2[:, 0] ** 2 + Etx2[:, 1] ** 2)).astype(np.float32)


def epiline_error(F, p1, p2):
    """float32 max of squared point-to-epiline distances in pixels (cv2 FMEstimatorCallback)."""
    x1 = np.c_[np.asarray(p1, np.float64), np.ones(len(p1))]
    x2 = np.c_[np.asarray(p2, np.float64), np.ones(len(p2))]
    l2 = x1 @ F.T  # epilines in image 2
    d2 = np.sum(x2 * l2, 1) ** 2 / (l2[:, 0] ** 2 + l2[:, 1] ** 2)
    l1 = x2 @ F
    d1 = np.sum(x1 * l1, 1) ** 2 / (l1[:, 0] ** 2 + l1[:, 1] ** 2)
    return np.maximum(d1, d2).astype(np.float32)


def inlier_mask(model, k1, k2, K, thr):
    if K is not None:
        t = thr / ((K[0, 0] + K[1, 1]) / 2)
        return sampson_error(model, normalize(k1, K), normalize(k2, K)) <= np.float32(t * t)
    return epiline_error(model, k1, k2) <= np.float32(thr * thr)


def skew(t):
    return np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])


def essential_from_pose(R, t):
    return skew(t) @ R


def fundamental_from_pose(R, t, K):
    Ki = np.linalg.inv(K)
    return Ki.T @ essential_from_pose(R, t) @ Ki


def _design(q1, q2):
    x1, y1 = q1[:, 0], q1[:, 1]
    x2, y2 = q2[:, 0], q2[:, 1]
    o = np.ones(len(q1))
    return np.stack([x2 * x1, x2 * y1, x2, y2 * x1, y2 * y1, y2, x1, y1, o], 1)


def _null(A, k):
    return np.linalg.svd(A)[2][-k:]


# --- 5-point: hidden-variable resultant (Li & Hartley) on dict polynomials ---------
def _pmul(a, b):
    out = {}
    for ea, ca in a.items():
        for eb, cb in b.items():
            e = (ea[0] + eb[0], ea[1] + eb[1], ea[2] + eb[2])
            out[e] = out.get(e, 0.0) + ca * cb
    return out


def _padd(a, b, s=1.0):
    out = dict(a)
    for e, c in b.items():
        out[e] = out.get(e, 0.0) + s * c
    return out


_XY = [(3, 0), (2, 1), (1, 2), (0, 3), (2, 0), (1, 1), (0, 2), (1, 0), (0, 1), (0, 0)]


def five_point(q1, q2):
    """All real essential matrices through 5 normalised correspondences (unit Frobenius)."""
    N = _null(_design(q1, q2), 4)  # rows X, Y, Z, W
    E = [{(1, 0, 0): N[0, k], (0, 1, 0): N[1, k], (0, 0, 1): N[2, k], (0, 0, 0): N[3, k]} for k in range(9)]
    eqs = []
    det = {}
    for sg, (a, b, c, d, e) in ((1, (0, 4, 8, 5, 7)), (-1, (1, 3, 8, 5, 6)), (1, (2, 3, 7, 4, 6))):
        det = _padd(det, _pmul(E[a], _padd(_pmul(E[b], E[c]), _pmul(E[d], E[e]), -1.0)), sg)
    eqs.append(det)
    EEt = [[None] * 3 for _ in range(3)]
    for i in range(3):
        for j in range(3):
            acc = {}
            for k in range(3):
                acc = _padd(acc, _pmul(E[i * 3 + k], E[j * 3 + k]))
            EEt[i][j] = acc
    tr = _padd(_padd(EEt[0][0], EEt[1][1]), EEt[2][2])
    for i in range(3):
        for j in range(3):
            acc = {}
            for k in range(3):
                a = EEt[i][k] if i != k else _padd(EEt[i][k], tr, -0.5)
                acc = _padd(acc, _pmul(a, E[k * 3 + j]))
            eqs.append(acc)

    def C_of(z):
        C = np.zeros((10, 10), dtype=np.result_type(z, np.float64))
        for r, eq in enumerate(eqs):
            for col, (a, b) in enumerate(_XY):
                C[r, col] = sum(eq.get((a, b, c), 0.0) * z ** c for c in range(4 - a - b))
        return C

    w = np.exp(2j * np.pi * np.arange(11) / 11)
    vals = np.array([np.linalg.det(C_of(z)) for z in w])
    coef = np.real(np.fft.fft(vals)) / 11.0  # coef[j] of z^j: vals[k] = sum_j coef[j] w_k^j
    roots = np.roots(coef[::-1])
    out = []
    for z in roots:
        if abs(z.imag) > 1e-8 * max(1.0, abs(z)):
            continue
        z = z.real
        m = np.linalg.svd(C_of(z))[2][-1]
        if abs(m[9]) < 1e-300:
            continue
        x, y = m[7] / m[9], m[8] / m[9]
        Ev = x * N[0] + y * N[1] + z * N[2] + N[3]
        out.append((Ev / np.linalg.norm(Ev)).reshape(3, 3))
    return out


def seven_point(q1, q2):
    """All real fundamental matrices through 7 correspondences (unit Frobenius)."""
    N = _null(_design(q1, q2), 2)
    F1, F2 = N[0].reshape(3, 3), N[1].reshape(3, 3)
    a = np.array([-1.0, 0.0, 1.0, 2.0])
    d = np.array([np.linalg.det(x * F1 + (1 - x) * F2) for x in a])
    c = np.polyfit(a, d, 3)
    out = []
    for r in np.roots(c):
        if abs(r.imag) > 1e-8 * max(1.0, abs(r)):
            continue
        F = r.real * F1 + (1 - r.real) * F2
        out.append(F / np.linalg.norm(F))
    return out


def decompose_essential(E):
    U, _, Vt = np.linalg.svd(E)
    if np.linalg.det(U) < 0:
        U = -U
    if np.linalg.det(Vt) < 0:
        Vt = -Vt
    W = np.array([[0.0, 1.0, 0.0], [-1.0, 0.0, 0.0], [0.0, 0.0, 1.0]])
    return U @ W @ Vt, U @ W.T @ Vt, U[:, 2].copy()


def _triangulate(P0, P1, p1, p2):
    X = []
    for (x1, y1), (x2, y2) in zip(p1, p2):
        A = np.stack([x1 * P0[2] - P0[0], y1 * P0[2] - P0[1], x2 * P1[2] - P1[0], y2 * P1[2] - P1[1]])
        X.append(np.linalg.svd(A)[2][-1])
    return np.array(X).T  # 4 x n


def recover_pose(E, k1, k2, K, dist=50.0):
    """cv2.recoverPose(E, k1, k2, K): returns (good, R, t)."""
    p1, p2 = normalize(k1, K), normalize(k2, K)
    R1, R2, t = decompose_essential(E)
    P0 = np.c_[np.eye(3), np.zeros(3)]
    goods = []
    for R, tt in ((R1, t), (R2, t), (R1, -t), (R2, -t)):
        P1 = np.c_[R, tt]
        Q = _triangulate(P0, P1, p1, p2)
        m = Q[2] * Q[3] > 0
        Q = Q / Q[3]
        m &= Q[2] < dist
        Q2 = P1 @ Q
        m &= (Q2[2] > 0) & (Q2[2] < dist)
        goods.append((int(m.sum()), R, tt))
    g = [x[0] for x in goods]
    if g[0] >= g[1] and g[0] >= g[2] and g[0] >= g[3]:
        return goods[0]
    if g[1] >= g[0] and g[1] >= g[2] and g[1] >= g[3]:
        return goods[1]
    if g[2] >= g[0] and g[2] >= g[1] and g[2] >= g[3]:
        return goods[2]
    return goods[3]


def rotation(axis, deg):
    axis = np.asarray(axis, np.float64)
    axis = axis / np.linalg.norm(axis)
    a = np.deg2rad(deg)
    Kx = skew(axis)
    return np.eye(3) + np.sin(a) * Kx + (1 - np.cos(a)) * Kx @ Kx


def synthetic_pair(rng, n_in, n_out, noise_px=0.5, K=ISEC_K, size=(720, 540), rot_deg=8.0, baseline=0.6):
    """Seeded two-view geometry: inliers from 3D points seen by both cameras (x2 = R x1 + t),
    outliers uniform in the image.  Returns k1, k2 (float32 [n, 2]), R, t (unit), is_inlier."""
    R = rotation(rng.normal(size=3), rot_deg)
    t = rng.normal(size=3)
    t = t / np.linalg.norm(t) * baseline
    w, h = size
    pts1, pts2 = [], []
    while len(pts1) < n_in:
        u = rng.uniform(0, w, 4 * n_in)
        v = rng.uniform(0, h, 4 * n_in)
        z = rng.uniform(2.0, 12.0, 4 * n_in)
        X = np.stack([(u - K[0, 2]) / K[0, 0] * z, (v - K[1, 2]) / K[1, 1] * z, z], 1)
        X2 = X @ R.T + t
        ok = X2[:, 2] > 0.5
        u2 = K[0, 0] * X2[:, 0] / X2[:, 2] + K[0, 2]
        v2 = K[1, 1] * X2[:, 1] / X2[:, 2] + K[1, 2]
        ok &= (u2 >= 0) & (u2 < w) & (v2 >= 0) & (v2 < h)
        for a, b, c, d in zip(u[ok], v[ok], u2[ok], v2[ok]):
            pts1.append((a, b))
            pts2.append((c, d))
    k1 = np.array(pts1[:n_in]) + rng.normal(0, noise_px, (n_in, 2))
    k2 = np.array(pts2[:n_in]) + rng.normal(0, noise_px, (n_in, 2))
    o1 = np.stack([rng.uniform(0, w, n_out), rng.uniform(0, h, n_out)], 1)
    o2 = np.stack([rng.uniform(0, w, n_out), rng.uniform(0, h, n_out)], 1)
    k1 = np.r_[k1, o1]
    k2 = np.r_[k2, o2]
    inl = np.r_[np.ones(n_in, bool), np.zeros(n_out, bool)]
    perm = rng.permutation(n_in + n_out)
    return (k1[perm].astype(np.float32), k2[perm].astype(np.float32), R, t / np.linalg.norm(t), inl[perm])


def rotation_angle_deg(Ra, Rb):
    c = (np.trace(Ra.T @ Rb) - 1) / 2
    return float(np.rad2deg(np.arccos(np.clip(c, -1, 1))))


# --- OpenCV's RANSAC loop (calib3d/ptsetreg.cpp RANSACPointSetRegistrator::run) ------
class CvRng:
    """cv::RNG: multiply-with-carry, state' = (uint32)state * 4164903690 + (state >> 32)."""

    def __init__(self, state=(1 << 64) - 1):
        self.state = state

    def next(self):
        s = self.state
        self.state = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & ((1 << 64) - 1)
        return self.state & 0xFFFFFFFF

    def uniform(self, a, b):
        return a if a == b else self.next() % (b - a) + a


def update_num_iters(p, ep, model_points, max_iters):
    """RANSACUpdateNumIters (ptsetreg.cpp); cvRound rounds half to even."""
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, np.finfo(np.float64).tiny)
    denom = 1.0 - (1.0 - ep) ** model_points
    if denom < np.finfo(np.float64).tiny:
        return 0
    num, denom = np.log(num), np.log(denom)
    return max_iters if (denom >= 0 or -num >= max_iters * (-denom)) else int(np.rint(num / denom))


def _collinear_last(pts):
    """haveCollinearPoints (fundam.cpp) for the last selected point (float32 coordinates)."""
    pts = np.asarray(pts, np.float32)
    i = len(pts) - 1
    for j in range(i):
        dx1, dy1 = float(pts[j, 0] - pts[i, 0]), float(pts[j, 1] - pts[i, 1])
        for k in range(j):
            dx2, dy2 = float(pts[k, 0] - pts[i, 0]), float(pts[k, 1] - pts[i, 1])
            if abs(dx2 * dy1 - dy2 * dx1) <= np.finfo(np.float32).eps * (abs(dx1) + abs(dy1) + abs(dx2) + abs(dy2)):
                return True
    return False


def cv_ransac(k1, k2, K=None, thr=3.0, confidence=0.999, max_iters=1000):
    """cv2.findEssentialMat(k1, k2, K, RANSAC, confidence, thr) when K is given, else
    cv2.findFundamentalMat(k1, k2, FM_RANSAC, thr, confidence) for >= 15 matches:
    OpenCV's sample stream (cv::RNG((uint64)-1), getSubset with duplicate redraw and,
    for F, the collinearity checkSubset), a model replaces the best iff its inlier
    count exceeds max(best, modelPoints - 1), each replacement shrinks the budget by
    RANSACUpdateNumIters.  Returns (model 3x3 or None, bool mask, inlier count)."""
    k1 = np.asarray(k1, np.float32)
    k2 = np.asarray(k2, np.float32)
    n = len(k1)
    if K is not None:
        m = 5
        p1, p2 = normalize(k1, K), normalize(k2, K)
        t = thr / ((K[0, 0] + K[1, 1]) / 2)
        t2 = np.float32(t * t)

        def solve(idx):
            return five_point(p1[idx], p2[idx])

        def err(M):
            return sampson_error(M, p1, p2)
    else:
        m = 7
        if n < 15:
            raise NotImplementedError("fewer than 15 matches: OpenCV switches FM_RANSAC to LMedS")
        t2 = np.float32(thr * thr)

        def solve(idx):
            return seven_point(k1[idx].astype(np.float64), k2[idx].astype(np.float64))

        def err(M):
            return epiline_error(M, k1, k2)
    if n < m:
        return None, np.zeros(n, bool), 0
    if n == m:
        sols = solve(np.arange(m))
        return (sols[0] if sols else None), np.ones(n, bool) if sols else np.zeros(n, bool), (n if sols else 0)
    rng = CvRng()
    niters, max_good, best, best_mask = max_iters, 0, None, np.zeros(n, bool)
    it = 0
    while it < niters:
        found = False
        for _attempt in range(10000):
            idx = []
            for _i in range(m):
                while True:
                    v = rng.uniform(0, n)
                    if v not in idx:
                        break
                idx.append(v)
            if m == 7 and (_collinear_last(k1[idx]) or _collinear_last(k2[idx])):
                continue
            found = True
            break
        if not found:
            break
        for M in solve(np.array(idx)):
            mask = err(M) <= t2
            g = int(mask.sum())
            if g > max(max_good, m - 1):
                max_good, best, best_mask = g, M, mask
                niters = update_num_iters(confidence, (n - g) / n, m, niters)
        it += 1
    if max_good == 0:
        return None, np.zeros(n, bool), 0
    return best, best_mask, max_good
