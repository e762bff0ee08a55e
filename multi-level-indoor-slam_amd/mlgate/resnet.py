"""ResNet-50 global descriptors on the GPU (``mlg_resnet50_forward``, include/mlgate.h):
the path MixVPR / SALAD actually execute in the reference, the torchvision ResNet-50
fallback of MixVPR._load_fallback_model / extract_descriptor
(scripts/semantic_gating/place_recognition.py:248-306).
"""
import numpy as np
import torch

from . import _native
from .weights import RESNET_STAGES, resolve_resnet50_state_dict

BN_EPS = 1e-5

BLOCK_ORDER = ("w1", "b1", "w2", "b2", "w3", "b3", "wd", "bd")  # mlg_rn_block field order


def fold_bn(w, sd, p):
    """Eval BatchNorm folded into the preceding conv: w * g / sqrt(v + eps), b - m * g / sqrt(v + eps)."""
    g = np.asarray(sd[p + ".weight"], np.float64)
    b = np.asarray(sd[p + ".bias"], np.float64)
    m = np.asarray(sd[p + ".running_mean"], np.float64)
    v = np.asarray(sd[p + ".running_var"], np.float64)
    sc = g / np.sqrt(v + BN_EPS)
    w = np.asarray(w, np.float64) * sc.reshape(-1, *([1] * (np.ndim(w) - 1)))
    return w.astype(np.float32), (b - m * sc).astype(np.float32)


class ResNet50GPU:
    """Batched ResNet-50 GAP descriptors, zero-padded / truncated to descriptor_dim."""

    def __init__(self, state_dict=None, device="cuda", weights_path=None, seed=0):
        self.device = _native.require_device(device)
        if state_dict is None:
            state_dict, self.weights_source = resolve_resnet50_state_dict(weights_path, seed)
        else:
            self.weights_source = "given"
        self._w = self._pack(state_dict)

    def _t(self, a, dtype):
        return torch.as_tensor(np.ascontiguousarray(a, np.float32)).to(dtype).contiguous().to(self.device)

    def _pack(self, sd):
        bf, f32 = torch.bfloat16, torch.float32
        sw, sb = fold_bn(sd["conv1.weight"], sd, "bn1")
        w = [self._t(sw.transpose(0, 2, 3, 1).reshape(64, 147), f32),  # [co][ky][kx][c]
             self._t(sb, f32)]
        empty = torch.empty(0, dtype=bf, device=self.device)
        cin, k = 64, 0
        for li, (width, blocks, _) in enumerate(RESNET_STAGES, 1):
            wpad = max(width, 128)
            for bi in range(blocks):
                p = f"layer{li}.{bi}."
                blk = {"wd": empty, "bd": empty.float()}
                w1, b1 = fold_bn(np.asarray(sd[p + "conv1.weight"]).reshape(width, cin), sd, p + "bn1")
                w2, b2 = fold_bn(sd[p + "conv2.weight"], sd, p + "bn2")
                w2 = w2.transpose(0, 2, 3, 1).reshape(width, 9 * width)  # k = tap * width + c
                pad = lambda a: np.concatenate([a, np.zeros((wpad - a.shape[0],) + a.shape[1:], np.float32)])  # noqa
                blk["w1"], blk["b1"] = self._t(pad(w1), bf), self._t(pad(b1[:, None])[:, 0], f32)
                blk["w2"], blk["b2"] = self._t(pad(w2), bf), self._t(pad(b2[:, None])[:, 0], f32)
                w3, b3 = fold_bn(np.asarray(sd[p + "conv3.weight"]).reshape(4 * width, width), sd, p + "bn3")
                blk["w3"], blk["b3"] = self._t(w3, bf), self._t(b3, f32)
                if bi == 0:
                    wd, bd = fold_bn(np.asarray(sd[p + "downsample.0.weight"]).reshape(4 * width, cin), sd,
                                     p + "downsample.1")
                    blk["wd"], blk["bd"] = self._t(wd, bf), self._t(bd, f32)
                w += [blk[f] for f in BLOCK_ORDER]
                cin = 4 * width
                k += 1
        return w

    def forward_device(self, frames, descriptor_dim):
        """frames: device uint8 [B, H, W, C] -> device f32 [B, descriptor_dim]."""
        if frames.dtype != torch.uint8:
            raise ValueError("frames must be uint8")
        if frames.dim() == 3:
            frames = frames[..., None]
        return _native.ops().resnet50(frames.contiguous(), self._w, int(descriptor_dim))
