"""LoFTR on the GPU: the detector-free matcher of the reference's ``LoFTR`` class
(scripts/semantic_gating/geometric_verification.py:424-526), which runs
``kornia.feature.LoFTR(pretrained='indoor')`` on grayscale frames (semantics: oracle/loftr.py).

``LoFTRGPU`` prepares the weights once (eval BatchNorm folded into the convs, the
196-channel stages zero-padded to 256, bf16 GEMM operands) and runs the backbone per
keyframe (``features``: cached by the caller, as every pair of a keyframe reuses it) and
the coarse / fine transformers and matching per batch of pairs (``match_device``) through
the ``torch.ops.mlgate.loftr_*`` operators (csrc/loftr.hip).  Weights: a kornia checkpoint
from ``MLGATE_LOFTR_WEIGHTS`` (torch.load, weights only), else seeded synthetic weights
(no network for the 'indoor' download).
"""
import functools

import numpy as np
import torch

from . import _native
from .weights import resolve_loftr_state_dict

D_C = 256
# (name, BatchNorm prefix or None, cin, cout) in mlg_loftr_weights.conv_w order
CONVS = (
    ("backbone.layer1.0.conv1", "backbone.layer1.0.bn1", 128, 128),
    ("backbone.layer1.0.conv2", "backbone.layer1.0.bn2", 128, 128),
    ("backbone.layer1.1.conv1", "backbone.layer1.1.bn1", 128, 128),
    ("backbone.layer1.1.conv2", "backbone.layer1.1.bn2", 128, 128),
    ("backbone.layer2.0.conv1", "backbone.layer2.0.bn1", 128, 196),
    ("backbone.layer2.0.conv2", "backbone.layer2.0.bn2", 196, 196),
    ("backbone.layer2.0.downsample.0", "backbone.layer2.0.downsample.1", 128, 196),
    ("backbone.layer2.1.conv1", "backbone.layer2.1.bn1", 196, 196),
    ("backbone.layer2.1.conv2", "backbone.layer2.1.bn2", 196, 196),
    ("backbone.layer3.0.conv1", "backbone.layer3.0.bn1", 196, 256),
    ("backbone.layer3.0.conv2", "backbone.layer3.0.bn2", 256, 256),
    ("backbone.layer3.0.downsample.0", "backbone.layer3.0.downsample.1", 196, 256),
    ("backbone.layer3.1.conv1", "backbone.layer3.1.bn1", 256, 256),
    ("backbone.layer3.1.conv2", "backbone.layer3.1.bn2", 256, 256),
    ("backbone.layer3_outconv", None, 256, 256),
    ("backbone.layer2_outconv", None, 196, 256),
    ("backbone.layer2_outconv2.0", "backbone.layer2_outconv2.1", 256, 256),
    ("backbone.layer2_outconv2.3", None, 256, 196),
    ("backbone.layer1_outconv", None, 128, 196),
    ("backbone.layer1_outconv2.0", "backbone.layer1_outconv2.1", 196, 196),
    ("backbone.layer1_outconv2.3", None, 196, 128),
)


def _pad(c):
    return 256 if c == 196 else c


def fold_bn(w, sd, bn, eps=1e-5):
    """conv weight [cout, cin, k, k] (+ eval BatchNorm) -> (weight, bias or None)."""
    if bn is None:
        return w, None
    g = sd[bn + ".weight"] / np.sqrt(sd[bn + ".running_var"] + np.float32(eps))
    return (w * g[:, None, None, None]).astype(np.float32), (sd[bn + ".bias"] - sd[bn + ".running_mean"] * g).astype(
        np.float32)


def pack_conv(w, cin_p, cout_p):
    """[cout, cin, k, k] -> [cout_p, k * k * cin_p] with column tap * cin_p + c (zero padded)."""
    cout, cin, k, _ = w.shape
    out = np.zeros((cout_p, k * k, cin_p), np.float32)
    out[:cout, :, :cin] = w.transpose(0, 2, 3, 1).reshape(cout, k * k, cin)
    return out.reshape(cout_p, k * k * cin_p)


@functools.lru_cache(maxsize=8)
def position_encoding(hc, wc, d=D_C):
    """PositionEncodingSine(d, temp_bug_fix=False) as [hc * wc, d] float32 (token = r * wc + c)."""
    y = np.cumsum(np.ones((hc, wc), np.float32), 0)[None]
    x = np.cumsum(np.ones((hc, wc), np.float32), 1)[None]
    div = np.exp(np.arange(0, d // 2, 2, dtype=np.float32) * np.float32(-np.log(10000.0) / d // 2))[:, None, None]
    pe = np.zeros((d, hc, wc), np.float32)
    pe[0::4] = np.sin(x * div)
    pe[1::4] = np.cos(x * div)
    pe[2::4] = np.sin(y * div)
    pe[3::4] = np.cos(y * div)
    return np.ascontiguousarray(pe.reshape(d, -1).T)


def weight_list(sd, device):
    """The torch.ops.mlgate.loftr_* weight tensor list (csrc/torch_ops.cpp loftr_weights)."""
    dev = torch.device(device)
    bf = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev).to(torch.bfloat16)  # noqa: E731
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    none = torch.empty(0, dtype=torch.float32, device=dev)
    w0, b0 = fold_bn(sd["backbone.conv1.weight"], sd, "backbone.bn1")
    out = [f32(w0.reshape(128, 49).T), f32(b0)]
    ws, bs = [], []
    for name, bn, cin, cout in CONVS:
        w, b = fold_bn(sd[name + ".weight"], sd, bn)
        ws.append(bf(pack_conv(w, _pad(cin), _pad(cout))))
        if b is None:
            bs.append(none)
        else:
            bp = np.zeros(_pad(cout), np.float32)
            bp[:cout] = b
            bs.append(f32(bp))
    out += ws + bs
    for pre, n in (("loftr_coarse", 8), ("loftr_fine", 2)):
        for i in range(n):
            p = f"{pre}.layers.{i}."
            out += [bf(np.concatenate([sd[p + "q_proj.weight"], sd[p + "k_proj.weight"], sd[p + "v_proj.weight"]])),
                    bf(sd[p + "merge.weight"]), bf(sd[p + "mlp.0.weight"]), bf(sd[p + "mlp.2.weight"]),
                    f32(sd[p + "norm1.weight"]), f32(sd[p + "norm1.bias"]), f32(sd[p + "norm2.weight"]),
                    f32(sd[p + "norm2.bias"])]
    mw = sd["fine_preprocess.merge_feat.weight"]
    out += [bf(sd["fine_preprocess.down_proj.weight"]), f32(sd["fine_preprocess.down_proj.bias"]), bf(mw[:, :128]),
            bf(mw[:, 128:]), f32(sd["fine_preprocess.merge_feat.bias"])]
    return out


class LoFTRGPU:
    """Batched LoFTR on device-resident keyframes."""

    def __init__(self, device="cuda", state_dict=None, seed=0, feature_batch=16):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise _native.MlgateError("LoFTR runs on the HIP device only (no CPU path)")
        if state_dict is None:
            state_dict, self.weights_source = resolve_loftr_state_dict(seed=seed)
        else:
            self.weights_source = "caller"
        self.ops = _native.ops()
        self.weights = weight_list(state_dict, self.device)
        # the fused coarse layer tails read their weights k-step packed: pack once here
        # (mlg_loftr_pack_tails), not on every mlg_loftr_match call
        self.weights.append(self.ops.loftr_pack_tails(self.weights))
        self.feature_batch = feature_batch
        self._pe = {}

    def features(self, frames):
        """uint8 [F, H, W, C] device frames -> (coarse [F, H8/8 W8/8, 256], fine [F, H8/2 W8/2, 128])
        f32 device tensors, H8 = H // 8 * 8 (other sizes go through cv2's gray + INTER_LINEAR
        resize on the device, as the reference resizes)."""
        outs = [self.ops.loftr_features(frames[i:i + self.feature_batch].contiguous(), self.weights)
                for i in range(0, frames.shape[0], self.feature_batch)]
        return torch.cat([c for c, _ in outs]), torch.cat([f for _, f in outs])

    def match_device(self, coarse, fine, H, W, pair_a, pair_b):
        """Pairs (pair_a[p], pair_b[p]) of feature rows -> device (counts [P], kpts0 / kpts1
        [P, L, 2], conf [P, L]); pair p's matches are the first counts[p] rows."""
        pa = torch.as_tensor(np.asarray(pair_a, np.int32))
        pb = torch.as_tensor(np.asarray(pair_b, np.int32))
        pe = self._pe.get((H, W))
        if pe is None:
            pe = self._pe[(H, W)] = torch.from_numpy(position_encoding(H // 8, W // 8)).to(self.device)
        return self.ops.loftr_match(coarse, fine, pa, pb, pe, self.weights, int(H), int(W))

    def match_frames(self, frames, pairs):
        """frames uint8 [F, H, W, C] (device), pairs [(a, b)] -> list of numpy (kpts0, kpts1, conf)
        in the pixel frame of the (H // 8 * 8, W // 8 * 8) resized gray image the model ran on."""
        pairs = list(pairs)
        if not pairs:
            return []
        H, W = int(frames.shape[1]) // 8 * 8, int(frames.shape[2]) // 8 * 8
        used = sorted({i for p in pairs for i in p})
        pos = {f: j for j, f in enumerate(used)}
        sel = frames[torch.as_tensor(used, device=frames.device)] if len(used) < frames.shape[0] else frames
        coarse, fine = self.features(sel)
        n, k0, k1, cf = self.match_device(coarse, fine, H, W, [pos[a] for a, _ in pairs], [pos[b] for _, b in pairs])
        n, k0, k1, cf = n.cpu().numpy(), k0.cpu().numpy(), k1.cpu().numpy(), cf.cpu().numpy()
        return [(k0[p, :n[p]], k1[p, :n[p]], cf[p, :n[p]]) for p in range(len(pairs))]
