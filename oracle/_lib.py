"""ctypes loader for oracle/build/liboracle.so (test infrastructure only)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(_HERE, "csrc", f) for f in ("oracle.c", "orb.c", "ransac_cv.c")]
        srcs.append(os.path.join(_HERE, "..", "multi-level-indoor-slam_amd", "csrc", "rs_math.h"))
        if not os.path.exists(_SO) or os.path.getmtime(_SO) < max(os.path.getmtime(f) for f in srcs if os.path.exists(f)):
            build()
        _lib = ctypes.CDLL(_SO)
        _lib.orc_resize_linear_u8.restype = ctypes.c_int
        _lib.orc_resize_vec_end.restype = ctypes.c_int
        _lib.orc_row_norms_f32.restype = ctypes.c_int
        _lib.orc_knn_rows.restype = ctypes.c_int
        _lib.orc_orb_detect.restype = ctypes.c_int
        _lib.orc_bf_match.restype = ctypes.c_int
        _lib.orc_five_point.restype = ctypes.c_int
        _lib.orc_essential_ransac.restype = ctypes.c_int
        _lib.orc_fundamental_ransac.restype = ctypes.c_int
        _lib.orc_rs_log.restype = ctypes.c_double
        _lib.orc_rs_log.argtypes = [ctypes.c_double]
        _lib.orc_rs_root.restype = ctypes.c_double
        _lib.orc_rs_root.argtypes = [ctypes.c_double, ctypes.c_int]
        _lib.orc_rs_update_iters.restype = ctypes.c_int
        _lib.orc_rs_update_iters.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int]
    return _lib


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def resize_linear_u8(img, dh, dw):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    c = 1 if img.ndim == 2 else img.shape[2]
    out = np.empty((dh, dw) + (() if img.ndim == 2 else (c,)), np.uint8)
    rc = lib().orc_resize_linear_u8(ptr(img), h, w, c, ptr(out), dh, dw)
    assert rc == 0
    return out


def row_norms_f32(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.shape[0], np.float32)
    lib().orc_row_norms_f32(ptr(x), ctypes.c_long(x.shape[0]), ctypes.c_long(x.shape[1]), ptr(out))
    return out


def knn_rows(S, q0, t, floor, has_floor, min_gap, thr, k, gating):
    S = np.ascontiguousarray(S, dtype=np.float32)
    Q, N = S.shape
    t = np.ascontiguousarray(t, dtype=np.float64)
    floor = np.ascontiguousarray(floor, dtype=np.int64)
    has_floor = np.ascontiguousarray(has_floor, dtype=np.uint8)
    kk = max(k, 1)
    idx = np.zeros((Q, kk), np.int32)
    sim = np.zeros((Q, kk), np.float32)
    valid = np.zeros((Q, kk), np.uint8)
    count = np.zeros(Q, np.int32)
    lib().orc_knn_rows(ptr(S), Q, N, q0, ptr(t), ptr(floor), ptr(has_floor), ctypes.c_double(min_gap),
                       ctypes.c_float(thr), k, int(gating), ptr(idx), ptr(sim), ptr(valid), ptr(count))
    return idx, sim, valid, count


def five_point(q1, q2):
    """oracle/csrc/ransac_cv.c orc_five_point: list of 3x3 essential matrices."""
    q1 = np.ascontiguousarray(q1, dtype=np.float64)
    q2 = np.ascontiguousarray(q2, dtype=np.float64)
    out = np.zeros((10, 9), np.float64)
    n = lib().orc_five_point(ptr(q1), ptr(q2), ptr(out))
    return [out[i].reshape(3, 3) for i in range(n)]


def essential_ransac(k1, k2, K, thr=3.0, confidence=0.999, max_iters=1000):
    """oracle/csrc/ransac_cv.c orc_essential_ransac: (model 3x3 or None, bool mask, inliers)."""
    k1 = np.ascontiguousarray(k1, dtype=np.float32)
    k2 = np.ascontiguousarray(k2, dtype=np.float32)
    Kc = np.ascontiguousarray(K, dtype=np.float64)
    n = len(k1)
    mask = np.zeros(max(n, 1), np.uint8)
    E = np.zeros(9, np.float64)
    g = lib().orc_essential_ransac(ptr(k1), ptr(k2), n, ptr(Kc), ctypes.c_double(thr), ctypes.c_double(confidence),
                                   max_iters, ptr(mask), ptr(E))
    return (E.reshape(3, 3) if E.any() else None), mask[:n].astype(bool), int(g)


def fundamental_ransac(k1, k2, thr=3.0, confidence=0.999, max_iters=1000, seed=0):
    """oracle/csrc/ransac_cv.c orc_fundamental_ransac: (model 3x3 or None, bool mask, inliers)."""
    k1 = np.ascontiguousarray(k1, dtype=np.float32)
    k2 = np.ascontiguousarray(k2, dtype=np.float32)
    n = len(k1)
    mask = np.zeros(max(n, 1), np.uint8)
    F = np.zeros(9, np.float64)
    g = lib().orc_fundamental_ransac(ptr(k1), ptr(k2), n, ctypes.c_double(thr), ctypes.c_double(confidence),
                                     max_iters, ctypes.c_uint64(int(seed) & ((1 << 63) - 1)), ptr(mask), ptr(F))
    return (F.reshape(3, 3) if F.any() else None), mask[:n].astype(bool), int(g)
