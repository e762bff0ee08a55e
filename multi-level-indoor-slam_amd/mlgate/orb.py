"""ORB + brute-force Hamming matching on the GPU: the reference's fallback matcher.

``LightGlue._load_fallback`` / ``_detect_and_match_fallback``
(geometric_verification.py:244-248, 314-350) run cv2.ORB_create(nfeatures=max_keypoints)
on BGR2GRAY frames and cv2.BFMatcher(NORM_HAMMING, crossCheck=True).match sorted by
distance.  Here both run as HIP kernels (csrc/orb.hip) over whole batches of frames and
pairs, through ``torch.ops.mlgate.orb_detect`` / ``orb_match``.

The ORB_Impl geometry is computed here, once per frame size: OpenCV's defaults
(scaleFactor 1.2, nlevels 8, edgeThreshold 31, patchSize 31, fastThreshold 20), level
sizes cvRound(cols / scale), nfeaturesPerLevel in float32, the u_max circle, the float32
Gaussian kernel of the per-level GaussianBlur(7x7, sigma 2), and the
point pattern: OpenCV's makeRandomPattern(31) stream (cv::RNG(0x34985739)) unless
MLGATE_ORB_PATTERN names an int [512, 2] .npy holding OpenCV's bit_pattern_31_ table
(not shipped: OpenCV is not installed here).  Deviations from OpenCV (parity unpinned):
see oracle/csrc/orb.c.
"""
import math
import os
from functools import lru_cache

import numpy as np

from . import _native

SCALE_FACTOR, NLEVELS, EDGE, PATCH, FAST_T = 1.2, 8, 31, 31, 20


@lru_cache(maxsize=None)
def geometry(H, W, nfeatures):
    """(int32 [42] block of mlg_orb_params: level widths, heights, features, umax[16],
    FAST threshold, edge threshold; float32 [15]: level scales, Gaussian kernel)."""
    f32 = np.float32
    scales = np.array([f32(np.power(np.float64(SCALE_FACTOR), l)) for l in range(NLEVELS)], np.float32)
    ws = [int(np.rint(f32(W) / s)) for s in scales]
    hs = [int(np.rint(f32(H) / s)) for s in scales]
    factor = f32(1.0 / SCALE_FACTOR)
    nd = f32(f32(nfeatures) * (f32(1) - factor) / (f32(1) - f32(np.power(np.float64(factor), NLEVELS))))
    per, total = [], 0
    for _ in range(NLEVELS - 1):
        n = int(np.rint(nd))
        per.append(n)
        total += n
        nd = f32(nd * factor)
    per.append(max(nfeatures - total, 0))
    half = PATCH // 2
    umax = [0] * (half + 2)
    vmax, vmin = int(np.floor(half * np.sqrt(2.0) / 2 + 1)), int(np.ceil(half * np.sqrt(2.0) / 2))
    for v in range(vmax + 1):
        umax[v] = int(np.rint(np.sqrt(float(half * half - v * v))))
    v0 = 0
    for v in range(half, vmin - 1, -1):
        while umax[v0] == umax[v0 + 1]:
            v0 += 1
        umax[v] = v0
        v0 += 1
    ip = ws + hs + per + umax[:16] + [FAST_T, EDGE]
    return np.array(ip, np.int32), np.concatenate([scales, gaussian_kernel()]).astype(np.float32)


def gaussian_kernel(ksize=7, sigma=2.0):
    """cv::getGaussianKernel(7, 2, CV_32F) as OpenCV 4.x builds it (getGaussianKernelBitExact:
    t_i = exp(x^2 * (-0.125 / sigma^2)) for x = 2 i - (n - 1), scaled by 1 / (2 sum t_i + 1),
    centre tap = that factor), rounded to float32 -- ORB's GaussianBlur(7x7, 2, 2)."""
    scale2 = -0.125 / (float(sigma) * float(sigma))
    n2 = (ksize - 1) // 2
    vals, s = [], 0.0
    for i in range(n2):
        x = 1 - ksize + 2 * i
        vals.append(math.exp(float(x * x) * scale2))
        s += vals[-1]
    mul1 = 1.0 / (s * 2.0 + 1.0)
    k = [mul1] * ksize
    for i in range(n2):
        k[i] = k[ksize - 1 - i] = vals[i] * mul1
    return np.array(k, np.float32)


def random_pattern(npoints=512):
    """OpenCV makeRandomPattern(31, pattern, 512): cv::RNG(0x34985739) multiply-with-carry,
    x then y = uniform(-15, 16) per point."""
    state = 0x34985739
    out = np.empty((npoints, 2), np.int16)
    for i in range(npoints):
        for c in range(2):
            state = ((state & 0xFFFFFFFF) * 4164903690 + (state >> 32)) & ((1 << 64) - 1)
            out[i, c] = (state & 0xFFFFFFFF) % 31 - 15
    return out


def load_pattern():
    path = os.environ.get("MLGATE_ORB_PATTERN")
    if path:
        pat = np.load(path, allow_pickle=False).astype(np.int16).reshape(512, 2)
        if np.abs(pat).max() > 15:
            raise ValueError(f"{path}: ORB pattern points must lie in [-15, 15]")
        return pat
    return random_pattern()


class OrbGPU:
    """Batched ORB detectAndCompute + cross-checked Hamming matching on the device."""

    def __init__(self, device="cuda", nfeatures=2048):
        import torch
        self.device = _native.require_device(device)
        self.nfeatures = int(nfeatures)
        self.max_kp = self.nfeatures + 256  # retainBest keeps ties at each level's cut
        self.pattern = torch.from_numpy(load_pattern().reshape(-1)).to(self.device)

    def detect_device(self, frames):
        """uint8 [F, H, W, C] device frames (BGR or gray) -> (kpts [F, K, 2], responses,
        angles, levels, descriptors [F, K, 32], counts [F]) device tensors."""
        import torch
        F, H, W = frames.shape[:3]
        ip, sc = geometry(int(H), int(W), self.nfeatures)
        out = _native.ops().orb_detect(frames.contiguous(), self.pattern, torch.from_numpy(ip),
                                       torch.from_numpy(sc), self.max_kp)
        cnt = out[5].cpu()
        if (cnt < 0).any():
            raise _native.MlgateError("orb_detect: a per-level candidate list overflowed")
        return out

    def match_device(self, desc, counts, pair_a, pair_b):
        """Cross-checked nearest neighbours per pair, sorted by distance (ties by query
        index): (query idx [P, K], train idx, distance, counts [P]) device tensors."""
        import torch
        dev = desc.device
        pa = torch.as_tensor(np.asarray(pair_a, np.int32), device=dev)
        pb = torch.as_tensor(np.asarray(pair_b, np.int32), device=dev)
        return _native.ops().orb_match(desc, counts, pa, pb)
