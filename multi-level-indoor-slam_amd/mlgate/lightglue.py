"""LightGlue matching on the GPU (``mlg_lightglue``, include/mlgate.h): the matcher half
of LightGlue._detect_and_match_native (scripts/semantic_gating/geometric_verification.py:
263-312) -- ``LightGlue(features='superpoint')`` with its defaults -- for a ragged batch
of keyframe pairs in one call.
"""
import numpy as np
import torch

from . import _native
from .weights import LG_LAYERS, resolve_lightglue_state_dict

PRUNING_MIN_KPTS_CUDA = 1536  # LightGlue.pruning_keypoint_thresholds['flash'] (CUDA + SDPA)
BLOCK_ORDER = ("Wqkv", "bqkv", "Wout", "bout", "Wf1", "bf1", "ln_g", "ln_b", "Wf2", "bf2")  # mlg_lg_block


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


def pack_rotary(ecos, esin):
    """Rotary factors cos / sin [Npad, 32] (token row, frequency) -> the projections' tile
    layout (csrc/common.h lg_fac4, include/mlgate.h mlg_op_lg_proj): [Npad / 64, 16, 64, 4]
    with (cos 2p, cos 2p + 1, sin 2p, sin 2p + 1) for row r, frequency pair p."""
    n = ecos.shape[0]
    cs = torch.stack([ecos.reshape(n // 64, 64, 16, 2), esin.reshape(n // 64, 64, 16, 2)], 3)  # [T, 64, 16, 2, 2]
    return cs.reshape(n // 64, 64, 16, 4).permute(0, 2, 1, 3).contiguous()


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
        self._w = self._pack(state_dict)

    def _t(self, a, dtype):
        return torch.as_tensor(np.ascontiguousarray(np.asarray(a, np.float32))).to(dtype).contiguous().to(self.device)

    def _pack(self, sd):
        """Device tensors in mlg_lg_weights order (torch.ops.mlgate.lightglue): Wr; the self
        then the cross blocks (BLOCK_ORDER each); final_proj weights, biases; matchability
        weights, biases; token-confidence weights, biases; a vector of ones."""
        bf, f32 = torch.bfloat16, torch.float32
        blocks = {"self": [], "cross": []}
        perm = qkv_row_order()
        for i in range(LG_LAYERS):
            p = f"transformers.{i}.self_attn."
            b = {"Wqkv": self._t(pack_kstep(np.asarray(sd[p + "Wqkv.weight"])[perm]), bf),
                 "bqkv": self._t(np.asarray(sd[p + "Wqkv.bias"])[perm], f32),
                 "Wout": self._t(pack_kstep(sd[p + "out_proj.weight"]), bf),
                 "bout": self._t(sd[p + "out_proj.bias"], f32)}
            blocks["self"].append(self._ffn(b, sd, p))
            p = f"transformers.{i}.cross_attn."
            c = {"Wqkv": self._t(pack_kstep(np.concatenate([sd[p + "to_qk.weight"], sd[p + "to_v.weight"]])), bf),
                 "bqkv": self._t(np.concatenate([sd[p + "to_qk.bias"], sd[p + "to_v.bias"]]), f32),
                 "Wout": self._t(pack_kstep(sd[p + "to_out.weight"]), bf),
                 "bout": self._t(sd[p + "to_out.bias"], f32)}
            blocks["cross"].append(self._ffn(c, sd, p))
        w = [self._t(sd["posenc.Wr.weight"], f32)]
        for kind in ("self", "cross"):
            for b in blocks[kind]:
                w += [b[f] for f in BLOCK_ORDER]
        la = [f"log_assignment.{i}." for i in range(LG_LAYERS)]
        tc = [f"token_confidence.{i}.token.0." for i in range(LG_LAYERS - 1)]
        w += [self._t(sd[p + "final_proj.weight"], bf) for p in la]
        w += [self._t(sd[p + "final_proj.bias"], f32) for p in la]
        w += [self._t(np.asarray(sd[p + "matchability.weight"]).reshape(-1), f32) for p in la]
        w += [self._t(np.asarray(sd[p + "matchability.bias"]).reshape(-1), f32) for p in la]
        w += [self._t(np.asarray(sd[p + "weight"]).reshape(-1), f32) for p in tc]
        w += [self._t(np.asarray(sd[p + "bias"]).reshape(-1), f32) for p in tc]
        w.append(self._t(np.ones(256, np.float32), f32))
        return w

    def _ffn(self, b, sd, p):
        bf, f32 = torch.bfloat16, torch.float32
        b["Wf1"], b["bf1"] = self._t(pack_kstep(sd[p + "ffn.0.weight"]), bf), self._t(sd[p + "ffn.0.bias"], f32)
        b["ln_g"], b["ln_b"] = self._t(sd[p + "ffn.1.weight"], f32), self._t(sd[p + "ffn.1.bias"], f32)
        b["Wf2"], b["bf2"] = self._t(pack_kstep(sd[p + "ffn.3.weight"]), bf), self._t(sd[p + "ffn.3.bias"], f32)
        return b

    def match_device(self, kpts, desc, counts, pair_a, pair_b):
        """kpts f32 [F, kmax, 2], desc f32 [F, kmax, 256] on the device; counts, pair_a, pair_b
        host int arrays.  Returns device (matches [P, kmax, 2], scores [P, kmax], num [P]) and the
        host stop layers [P]."""
        kmax = int(kpts.shape[1])
        if kmax > 2048:
            raise ValueError(f"LightGlue supports up to 2048 keypoints per image (got {kmax})")
        host = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.int32)))  # noqa: E731
        m, s, n, stop = _native.ops().lightglue(kpts.contiguous(), desc.contiguous(), host(counts), host(pair_a),
                                                host(pair_b), self._w, self.depth_confidence, self.width_confidence,
                                                self.filter_threshold, self.pruning_min_kpts)
        return m, s, n, stop.numpy()

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
