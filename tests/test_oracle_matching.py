"""CPU sanity checks of the SuperPoint and LightGlue oracles (oracle/superpoint.py,
oracle/lightglue.py) -- the checkers the GPU parity tests compare against."""
import numpy as np
import torch

from mlgate.weights import lightglue_state_dict, superpoint_state_dict
from oracle import lightglue as olg
from oracle import superpoint as osp


def test_gray_conversion_matches_cv2_fixed_point():
    img = np.array([[[0, 0, 0], [255, 255, 255], [10, 200, 30], [255, 0, 0], [0, 0, 255]]], np.uint8)
    g = osp.bgr_to_gray_u8(img)[0]
    # cv2: (1868 B + 9617 G + 4899 R + 8192) >> 14
    assert list(g) == [0, 255, (10 * 1868 + 200 * 9617 + 30 * 4899 + 8192) >> 14, 29, 76]


def test_simple_nms_keeps_isolated_maxima():
    s = torch.zeros(1, 32, 32)
    s[0, 5, 5], s[0, 5, 8], s[0, 20, 20] = 0.9, 0.5, 0.7
    out = osp.simple_nms(s, 4)
    assert out[0, 5, 5] == 0.9 and out[0, 20, 20] == 0.7 and out[0, 5, 8] == 0


def test_superpoint_oracle_shapes_and_order():
    sd = superpoint_state_dict(0)
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (64, 96, 3), dtype=np.uint8)
    r = osp.superpoint(sd, [img], max_kp=50)[0]
    assert r["keypoints"].shape == (50, 2) and r["descriptors"].shape == (50, 256)
    assert torch.all(r["keypoint_scores"][:-1] >= r["keypoint_scores"][1:])
    assert torch.allclose(r["descriptors"].norm(dim=1), torch.ones(50), atol=1e-5)
    r = osp.superpoint(sd, [img], max_kp=100000)[0]  # all kept -> raster order
    ras = r["keypoints"][:, 1] * 96 + r["keypoints"][:, 0]
    assert torch.all(ras[1:] > ras[:-1])


def test_lightglue_oracle_matches_synthetic_correspondences():
    rng = np.random.default_rng(1)
    m, n, no = 300, 280, 200
    k0 = np.stack([rng.uniform(0, 640, m), rng.uniform(0, 480, m)], 1).astype(np.float32)
    d0 = rng.standard_normal((m, 256)).astype(np.float32)
    d0 /= np.linalg.norm(d0, axis=1, keepdims=True)
    k1 = np.stack([rng.uniform(0, 640, n), rng.uniform(0, 480, n)], 1).astype(np.float32)
    d1 = rng.standard_normal((n, 256)).astype(np.float32)
    k1[:no] = k0[:no] + 10
    d1[:no] = d0[:no] + 0.02 * rng.standard_normal((no, 256))
    d1 /= np.linalg.norm(d1, axis=1, keepdims=True)
    r = olg.Oracle(lightglue_state_dict(0)).match(k0, d0, k1, d1)
    mt = r["matches"].numpy()
    assert len(mt) > 0.8 * no
    assert np.mean(mt[:, 0] == mt[:, 1]) > 0.9
    assert np.all(np.diff(mt[:, 0]) > 0)
    assert 1 <= r["stop"] <= 9


def test_confidence_thresholds():
    assert olg.conf_threshold(0) == 0.9
    assert abs(olg.conf_threshold(8) - (0.8 + 0.1 * np.exp(-32 / 9))) < 1e-12
