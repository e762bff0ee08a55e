"""Oracle for the LiDAR floor tracker's per-scan compute (test infrastructure only).

Restates LiDARFloorTracker.extract_ground_points / fit_ground_plane_ransac
(scripts/semantic_gating/lidar_floor_tracker.py:70-141) in numpy with a pluggable
3-point sampler: ``numpy_sampler`` is the reference's own (np.random.choice, unseeded
in the reference, seeded here), ``counter_sampler`` restates the GPU kernel's
counter-based stream (csrc/plane.hip) so plane parameters and inlier counts can be
compared exactly.  Parity of the reference's numbers is decision-level (its RNG is
unseeded, so no fixture can pin the planes themselves).
"""
import numpy as np

M64 = (1 << 64) - 1


def _mix(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def counter_sampler(seed=0):
    def sample(h, n):
        st = _mix((seed ^ ((h * 0x632BE59BD9B4E019) & M64)) & M64)
        idx = []
        while len(idx) < 3:
            st = _mix(st)
            v = (st >> 11) % n
            if v not in idx:
                idx.append(v)
        return np.array(idx)
    return sample


def numpy_sampler(seed=0):
    rng = np.random.default_rng(seed)
    return lambda h, n: rng.choice(n, 3, replace=False)


def extract_ground_points(points, rings=None, ring_threshold=30):
    if rings is not None:
        return points[rings < ring_threshold]
    z_min = np.percentile(points[:, 2], 5)
    return points[points[:, 2] < (z_min + 0.5)]


def fit_ground_plane(points, iterations=100, threshold=0.1, sampler=None):
    """-> (plane [a, b, c, d] or None, inlier_ratio, best_inliers); float64 math on the points."""
    if len(points) < 3:
        return None, 0.0, 0
    sampler = sampler or counter_sampler(0)
    P = np.asarray(points, np.float64)
    best, best_n = None, 0
    for h in range(iterations):
        i = sampler(h, len(P))
        p1, p2, p3 = P[i]
        v1, v2 = p2 - p1, p3 - p1
        nrm = np.array([v1[1] * v2[2] - v1[2] * v2[1], v1[2] * v2[0] - v1[0] * v2[2], v1[0] * v2[1] - v1[1] * v2[0]])
        ln = np.sqrt(nrm @ nrm)
        if ln < 1e-6:
            continue
        nrm = nrm / ln
        d = -(nrm[0] * p1[0] + nrm[1] * p1[1] + nrm[2] * p1[2])
        dist = np.abs((P[:, 0] * nrm[0] + P[:, 1] * nrm[1]) + P[:, 2] * nrm[2] + d)
        n_in = int(np.sum(dist < threshold))
        if n_in > best_n:
            best_n, best = n_in, np.array([nrm[0], nrm[1], nrm[2], d])
    return best, best_n / len(P), best_n


def synthetic_scans(rng, n_scans, floors, floor_height=3.5, n_ground=900, n_clutter=300):
    """Scans whose ground plane sits at -1.5 + floor * floor_height (slightly tilted), with
    clutter above it; returns (points list, timestamps)."""
    out = []
    for f in floors[:n_scans]:
        x = rng.uniform(-10, 10, n_ground)
        y = rng.uniform(-10, 10, n_ground)
        z = -1.5 + f * floor_height + 0.01 * x - 0.005 * y + rng.normal(0, 0.03, n_ground)
        g = np.stack([x, y, z], 1)
        c = np.stack([rng.uniform(-10, 10, n_clutter), rng.uniform(-10, 10, n_clutter),
                      -1.5 + f * floor_height + rng.uniform(0.6, 3.0, n_clutter)], 1)
        out.append(np.concatenate([g, c]).astype(np.float32))
    return out, np.arange(len(out)) * 0.5
