"""ORB + BFMatcher fallback matcher, CPU restatement (TEST INFRASTRUCTURE ONLY).

Reference: geometric_verification.py:244-248 (cv2.ORB_create(nfeatures=max_keypoints),
cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True)) and :314-350
(_detect_and_match_fallback).  The per-pixel / per-keypoint work is in
oracle/csrc/orb.c (see its header for what is restated and what is unpinned); this
module restates the ORB_Impl geometry (OpenCV orb.cpp defaults: scaleFactor 1.2,
nlevels 8, edgeThreshold 31, patchSize 31, fastThreshold 20, WTA_K 2, HARRIS_SCORE)
and the reference's Python around the two OpenCV calls.
"""
import ctypes
import math

import numpy as np

from . import _lib
from .geometry import CvRng

SCALE_FACTOR, NLEVELS, EDGE, PATCH, FAST_T = 1.2, 8, 31, 31, 20


def level_geometry(H, W, nfeatures, scale_factor=SCALE_FACTOR, nlevels=NLEVELS):
    """(scales float32 [L], widths [L], heights [L], features per level [L]).

    ORB_Impl: scale = (float)pow(scaleFactor, level); size = cvRound(cols / scale);
    ndesired = nfeatures * (1 - factor) / (1 - factor^nlevels) with factor = 1 / 1.2,
    cvRound per level, the remainder on the last level (all float32 arithmetic)."""
    f32 = np.float32
    scales = np.array([f32(np.power(np.float64(scale_factor), l)) for l in range(nlevels)], np.float32)
    ws = np.array([int(np.rint(f32(W) / s)) for s in scales], np.int32)
    hs = np.array([int(np.rint(f32(H) / s)) for s in scales], np.int32)
    factor = f32(1.0 / scale_factor)
    nd = f32(f32(nfeatures) * (f32(1) - factor) / (f32(1) - f32(np.power(np.float64(factor), nlevels))))
    per, total = [], 0
    for _ in range(nlevels - 1):
        n = int(np.rint(nd))
        per.append(n)
        total += n
        nd = f32(nd * factor)
    per.append(max(nfeatures - total, 0))
    return scales, ws, hs, np.array(per, np.int32)


def random_pattern(npoints=512, patch=PATCH):
    """OpenCV makeRandomPattern(patchSize, pattern, npoints): cv::RNG(0x34985739),
    x then y = rng.uniform(-patch/2, patch/2 + 1) per point -> int32 [npoints, 2]."""
    rng = CvRng(0x34985739)
    half = patch // 2
    pts = np.empty((npoints, 2), np.int32)
    for i in range(npoints):
        for c in range(2):
            u = rng.next() % (2 * half + 1)
            pts[i, c] = u - half
    return pts


def umax_table(half=PATCH // 2):
    """ORB_Impl's u_max circle rows (orb.cpp)."""
    umax = np.zeros(half + 2, np.int32)
    vmax = int(np.floor(half * np.sqrt(2.0) / 2 + 1))
    vmin = int(np.ceil(half * np.sqrt(2.0) / 2))
    for v in range(vmax + 1):
        umax[v] = int(np.rint(np.sqrt(float(half * half - v * v))))
    v0 = 0
    for v in range(half, vmin - 1, -1):
        while umax[v0] == umax[v0 + 1]:
            v0 += 1
        umax[v] = v0
        v0 += 1
    return umax


def gauss_kernel(ksize=7, sigma=2.0):
    """cv::getGaussianKernel(ksize, sigma, CV_32F) of OpenCV 4.x: getGaussianKernelBitExact
    (x = 2 i - (n - 1), t_i = exp(x^2 * (-0.125 / sigma^2)), normaliser 1 / (2 sum t_i + 1),
    centre = the normaliser) rounded to float32."""
    scale2 = -0.125 / (float(sigma) * float(sigma))
    n2 = (ksize - 1) // 2
    vals, s = [], 0.0
    for i in range(n2):
        x = 1 - ksize + 2 * i
        t = math.exp(float(x * x) * scale2)
        vals.append(t)
        s += t
    mul1 = 1.0 / (s * 2.0 + 1.0)
    k = [mul1] * ksize
    for i in range(n2):
        k[i] = k[ksize - 1 - i] = vals[i] * mul1
    return np.array(k, np.float32)


def resize_exact(img, DH, DW):
    """cv::resize(img, (DW, DH), INTER_LINEAR_EXACT) on one 8-bit channel (orb.c)."""
    img = np.ascontiguousarray(img, np.uint8)
    out = np.empty((DH, DW), np.uint8)
    _lib.lib().orc_resize_exact_u8(_lib.ptr(img), img.shape[0], img.shape[1], _lib.ptr(out), DH, DW)
    return out


def blur(img):
    """ORB's GaussianBlur(7x7, 2, 2, BORDER_REFLECT_101) of one level (orb.c)."""
    img = np.ascontiguousarray(img, np.uint8)
    out = np.empty_like(img)
    k = gauss_kernel()
    _lib.lib().orc_gauss7(_lib.ptr(img), img.shape[0], img.shape[1], _lib.ptr(k), _lib.ptr(out))
    return out


def gray(img):
    """cv2.cvtColor(BGR2GRAY) on uint8 (OpenCV's 14-bit fixed-point weights)."""
    img = np.asarray(img)
    if img.ndim == 2:
        return np.ascontiguousarray(img, np.uint8)
    b, g, r = (img[..., i].astype(np.int32) for i in range(3))
    return ((b * 1868 + g * 9617 + r * 4899 + 8192) >> 14).astype(np.uint8)


def detect_and_compute(gray_img, nfeatures, pattern=None):
    """ORB detectAndCompute -> (kpts float32 [n, 2] level-0 (x, y), levels, responses,
    angles (degrees), descriptors uint8 [n, 32])."""
    g = np.ascontiguousarray(gray_img, np.uint8)
    H, W = g.shape
    scales, ws, hs, per = level_geometry(H, W, nfeatures)
    pat = np.ascontiguousarray(random_pattern() if pattern is None else pattern, np.int32)
    um, gk = umax_table(), gauss_kernel()
    cap = int(per.sum()) * 4 + 64
    kx, ky, kr, ka = (np.zeros(cap, np.float32) for _ in range(4))
    kl = np.zeros(cap, np.int32)
    kd = np.zeros((cap, 32), np.uint8)
    p = _lib.ptr
    n = _lib.lib().orc_orb_detect(p(g), H, W, NLEVELS, p(ws), p(hs), p(scales), p(per), p(pat), p(um), p(gk),
                                  FAST_T, EDGE, p(kx), p(ky), p(kl), p(kr), p(ka), p(kd), cap)
    assert n >= 0
    return np.stack([kx[:n], ky[:n]], 1), kl[:n], kr[:n], ka[:n], kd[:n]


def bf_match(d1, d2):
    """BFMatcher(NORM_HAMMING, crossCheck=True).match + sorted(key=distance) ->
    (query idx, train idx, distance) int32 arrays."""
    d1 = np.ascontiguousarray(d1, np.uint8)
    d2 = np.ascontiguousarray(d2, np.uint8)
    n = max(len(d1), 1)
    qi, ti, dist = (np.zeros(n, np.int32) for _ in range(3))
    p = _lib.ptr
    m = _lib.lib().orc_bf_match(p(d1), ctypes.c_int(len(d1)), p(d2), ctypes.c_int(len(d2)), p(qi), p(ti), p(dist))
    return qi[:m], ti[:m], dist[:m]


def detect_and_match_fallback(image1, image2, max_keypoints=2048, pattern=None):
    """geometric_verification.py:314-350 with the ORB / BFMatcher restatements."""
    k1, _, _, _, d1 = detect_and_compute(gray(image1), max_keypoints, pattern)
    k2, _, _, _, d2 = detect_and_compute(gray(image2), max_keypoints, pattern)
    if len(d1) == 0 or len(d2) == 0 or len(k1) < 5 or len(k2) < 5:
        return np.array([]), np.array([]), np.array([])
    qi, ti, dist = bf_match(d1, d2)
    m1 = np.array([k1[i].tolist() for i in qi])
    m2 = np.array([k2[j].tolist() for j in ti])
    max_dist = max(float(d) for d in dist) if len(dist) else 1
    conf = np.array([1 - float(d) / max_dist for d in dist])
    return m1, m2, conf
