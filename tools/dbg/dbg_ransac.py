import sys, numpy as np
sys.path.insert(0, "multi-level-indoor-slam_amd"); sys.path.insert(0, ".")
from mlgate import geometry
from oracle import geometry as G
rng = np.random.default_rng(2)
k1, k2, R, t, inl = G.synthetic_pair(rng, 300, 100, 0.5)
for H in (1, 2, 3, 4, 5, 6, 7, 8, 64, 1024):
    r = geometry.epipolar_ransac([k1], [k2], None, 3.0, hypotheses=H)[0]
    print(H, r.inliers, r.status)
