"""LightGlue matching on the GPU (``mlg_lightglue``, include/mlgate.h): the matcher half
of LightGlue._detect_and_match_native (scripts/semantic_gating/geometric_verification.py:
263-312) -- ``LightGlue(features='superpoint')`` with its defaults -- for a ragged batch
of keyframe pairs in one call.
"""
import ctypes

import numpy as np
import torch

from . import _native
from .weights import LG_LAYERS, resolve_lightglue_state_dict

PRUNING_MIN_KPTS_CUDA = 1536  # LightGlue.pruning_keypoint_thresholds['flash'] (CUDA + SDPA)


class _Block(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("Wqkv", "bqkv", "Wout", "bout", "Wf1", "bf1", "ln_g", "ln_b", "Wf2",
                                               "bf2")]


class _Weights(ctypes.Structure):
    _fields_ = [("Wr", ctypes.c_void_p), ("self_", _Block * 9), ("cross", _Block * 9),
                ("Wfinal", ctypes.c_void_p * 9), ("bfinal", ctypes.c_void_p * 9),
                ("wmatch", ctypes.c_void_p * 9), ("bmatch", ctypes.c_void_p * 9),
                ("wconf", ctypes.c_void_p * 8), ("bconf", ctypes.c_void_p * 8), ("ones", ctypes.c_void_p)]


def qkv_row_order():
    """Row permutation of SelfBlock.Wqkv from the reference's (head, 64, 3) interleave
    (``qkv.unflatten(-1, (heads, -1, 3))``) to [q | k | v] x (head, dim), the layout the
    projection kernel expects (csrc/lg_proj.hip: parts q, k, v of 256 columns each)."""
    s, h, d = np.meshgrid(np.arange(3), np.arange(4), np.arange(64), indexing="ij")
    return (h * 192 + d * 3 + s).reshape(-1)


def pack_kstep(w):
    """nn.Linear weight [N, K] -> k-step-major [K/16, N, 16] (the layout of the fused
    block-tail and projection kernels, csrc/lg_ffn.hip / lg_proj.hip: a wave's 32 rows x
    16 k of one MFMA step are one contiguous 1 KiB)."""
    w = np.asarray(w, np.float32)
    n, k = w.shape
    return np.ascontiguousarray(w.reshape(n, k // 16, 16).transpose(1, 0, 2))


class LightGlueGPU:
    """Batched LightGlue(features='superpoint') on the HIP device."""

    def __init__(self, state_dict=None, device="cuda", depth_confidence=0.95, width_confidence=0.99,
                 filter_threshold=0.1, pruning_min_kpts=PRUNING_MIN_KPTS_CUDA, weights_path=None, seed=0):
        self.device = _native.require_device(device)
        if state_dict is None:
            state_dict, self.weights_source = resolve_lightglue_state_dict(weights_path, seed)
        else:
            self.weights_source = "given"
        self.depth_confidence = float(depth_confidence)
        self.width_confidence = float(width_confidence)
        self.filter_threshold = float(filter_threshold)
        self.pruning_min_kpts = int(pruning_min_kpts)
        self._keep = []
        self._w = self._pack(state_dict)
        self._ws = None

    def _t(self, a, dtype):
        t = torch.as_tensor(np.ascontiguousarray(np.asarray(a, np.float32))).to(dtype).contiguous().to(self.device)
        self._keep.append(t)
        return t.data_ptr()

    def _pack(self, sd):
        bf, f32 = torch.bfloat16, torch.float32
        w = _Weights()
        w.Wr = self._t(sd["posenc.Wr.weight"], f32)
        for i in range(LG_LAYERS):
            p = f"transformers.{i}.self_attn."
            b = w.self_[i]
            perm = qkv_row_order()
            b.Wqkv = self._t(pack_kstep(np.asarray(sd[p + "Wqkv.weight"])[perm]), bf)
            b.bqkv = self._t(np.asarray(sd[p + "Wqkv.bias"])[perm], f32)
            b.Wout = self._t(pack_kstep(sd[p + "out_proj.weight"]), bf)
            b.bout = self._t(sd[p + "out_proj.bias"], f32)
            self._ffn(b, sd, p)
            p = f"transformers.{i}.cross_attn."
            c = w.cross[i]
            c.Wqkv = self._t(pack_kstep(np.concatenate([sd[p + "to_qk.weight"], sd[p + "to_v.weight"]])), bf)
            c.bqkv = self._t(np.concatenate([sd[p + "to_qk.bias"], sd[p + "to_v.bias"]]), f32)
            c.Wout = self._t(pack_kstep(sd[p + "to_out.weight"]), bf)
            c.bout = self._t(sd[p + "to_out.bias"], f32)
            self._ffn(c, sd, p)
            p = f"log_assignment.{i}."
            w.Wfinal[i] = self._t(sd[p + "final_proj.weight"], bf)
            w.bfinal[i] = self._t(sd[p + "final_proj.bias"], f32)
            w.wmatch[i] = self._t(np.asarray(sd[p + "matchability.weight"]).reshape(-1), f32)
            w.bmatch[i] = self._t(np.asarray(sd[p + "matchability.bias"]).reshape(-1), f32)
            if i < LG_LAYERS - 1:
                p = f"token_confidence.{i}.token.0."
                w.wconf[i] = self._t(np.asarray(sd[p + "weight"]).reshape(-1), f32)
                w.bconf[i] = self._t(np.asarray(sd[p + "bias"]).reshape(-1), f32)
        w.ones = self._t(np.ones(256, np.float32), f32)
        return w

    def _ffn(self, b, sd, p):
        bf, f32 = torch.bfloat16, torch.float32
        b.Wf1, b.bf1 = self._t(pack_kstep(sd[p + "ffn.0.weight"]), bf), self._t(sd[p + "ffn.0.bias"], f32)
        b.ln_g, b.ln_b = self._t(sd[p + "ffn.1.weight"], f32), self._t(sd[p + "ffn.1.bias"], f32)
        b.Wf2, b.bf2 = self._t(pack_kstep(sd[p + "ffn.3.weight"]), bf), self._t(sd[p + "ffn.3.bias"], f32)

    def match_device(self, kpts, desc, counts, pair_a, pair_b):
        """kpts f32 [F, kmax, 2], desc f32 [F, kmax, 256] on the device; counts, pair_a, pair_b
        host int arrays.  Returns device (matches [P, kmax, 2], scores [P, kmax], num [P]) and the
        host stop layers [P]."""
        F, kmax = int(kpts.shape[0]), int(kpts.shape[1])
        counts = np.ascontiguousarray(np.asarray(counts, np.int32))
        pa = np.ascontiguousarray(np.asarray(pair_a, np.int32))
        pb = np.ascontiguousarray(np.asarray(pair_b, np.int32))
        P = len(pa)
        L = _native.lib()
        nbytes = L.mlg_lightglue_workspace_bytes(P, kmax)
        if nbytes == 0:
            raise ValueError(f"LightGlue supports up to 2048 keypoints per image (got {kmax})")
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        m = torch.empty(P, kmax, 2, dtype=torch.int32, device=self.device)
        s = torch.empty(P, kmax, dtype=torch.float32, device=self.device)
        n = torch.empty(P, dtype=torch.int32, device=self.device)
        stop = np.zeros(P, np.int32)
        i32p = ctypes.POINTER(ctypes.c_int32)
        rc = L.mlg_lightglue(ctypes.byref(self._w), _native.ptr(kpts.contiguous()), _native.ptr(desc.contiguous()),
                             counts.ctypes.data_as(i32p), F, kmax, pa.ctypes.data_as(i32p), pb.ctypes.data_as(i32p), P,
                             self.depth_confidence, self.width_confidence, self.filter_threshold,
                             self.pruning_min_kpts, _native.ptr(self._ws), self._ws.numel(), _native.ptr(m),
                             _native.ptr(s), _native.ptr(n), stop.ctypes.data_as(i32p), _native.stream_of(self.device))
        _native.check(rc, "mlg_lightglue")
        return m, s, n, stop

    def match(self, feats0, feats1):
        """Host convenience for one pair of SuperPoint outputs (dicts of numpy arrays):
        returns (matches [S, 2], scores [S], stop)."""
        k = max(len(feats0["keypoints"]), len(feats1["keypoints"]), 1)
        kp = torch.zeros(2, k, 2, dtype=torch.float32)
        ds = torch.zeros(2, k, 256, dtype=torch.float32)
        for j, f in enumerate((feats0, feats1)):
            nk = len(f["keypoints"])
            kp[j, :nk] = torch.as_tensor(np.asarray(f["keypoints"], np.float32))
            ds[j, :nk] = torch.as_tensor(np.asarray(f["descriptors"], np.float32))
        counts = [len(feats0["keypoints"]), len(feats1["keypoints"])]
        m, s, n, stop = self.match_device(kp.to(self.device), ds.to(self.device), counts, [0], [1])
        c = int(n[0])
        return m[0, :c].cpu().numpy(), s[0, :c].cpu().numpy(), int(stop[0])
