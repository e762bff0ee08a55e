"""SuperPoint on the GPU (``mlg_superpoint``, include/mlgate.h): the extractor half of
LightGlue._detect_and_match_native (scripts/semantic_gating/geometric_verification.py:
263-312) -- ``SuperPoint(max_num_keypoints=2048, detection_threshold=0.001)`` on
``cv2.cvtColor(img, COLOR_BGR2GRAY) / 255`` -- for a batch of keyframes at once.
"""
import numpy as np
import torch

from . import _native
from .weights import SUPERPOINT_LAYERS, resolve_superpoint_state_dict

DESC_DIM = 256
_ORDER = ["conv1b", "conv2a", "conv2b", "conv3a", "conv3b", "conv4a", "conv4b", "convPa", "convPb", "convDa",
          "convDb"]



def pack_weights(sd, device):
    """Device tensors in the kernel layouts: bf16 [Cout][3][3][Cin] / [Cout][Cin]; convPb padded to 128 rows."""
    t = {}
    w1 = torch.as_tensor(np.asarray(sd["conv1a.weight"], np.float32)).reshape(64, 9)
    t["conv1a.w"] = w1.contiguous().to(device)
    t["conv1a.b"] = torch.as_tensor(np.asarray(sd["conv1a.bias"], np.float32)).to(device)
    for name, cin, cout, k in SUPERPOINT_LAYERS[1:]:
        w = torch.as_tensor(np.asarray(sd[f"{name}.weight"], np.float32))
        b = torch.as_tensor(np.asarray(sd[f"{name}.bias"], np.float32))
        w = w.permute(0, 2, 3, 1).reshape(cout, k * k * cin)
        if name == "convPb":
            w = torch.cat([w, torch.zeros(128 - cout, w.shape[1])])
            b = torch.cat([b, torch.zeros(128 - cout)])
        t[f"{name}.w"] = w.to(torch.bfloat16).contiguous().to(device)
        t[f"{name}.b"] = b.contiguous().to(device)
    return t


class SuperPointGPU:
    """Batched SuperPoint keypoints / descriptors on the HIP device."""

    def __init__(self, state_dict=None, device="cuda", max_num_keypoints=2048, detection_threshold=0.001,
                 nms_radius=4, remove_borders=4, weights_path=None, seed=0):
        self.device = _native.require_device(device)
        if state_dict is None:
            state_dict, self.weights_source = resolve_superpoint_state_dict(weights_path, seed)
        else:
            self.weights_source = "given"
        self.max_kp = int(max_num_keypoints)
        self.det_thr = float(detection_threshold)
        self.nms_radius = int(nms_radius)
        self.border = int(remove_borders)
        self._t = pack_weights(state_dict, self.device)
        # mlg_sp_weights order: conv1a w, b; the 11 bf16 weights; their 11 biases
        self._w = ([self._t["conv1a.w"], self._t["conv1a.b"]] + [self._t[f"{n}.w"] for n in _ORDER]
                   + [self._t[f"{n}.b"] for n in _ORDER])

    def extract_device(self, frames, with_bf16=False):
        """frames: device uint8 [B, H, W, C] -> device (kpts [B, K, 2], scores [B, K], desc [B, K, 256],
        desc_bf16 or None, counts [B])."""
        if frames.dtype != torch.uint8 or frames.dim() not in (3, 4):
            raise ValueError("frames must be uint8 [B, H, W, C] or [B, H, W]")
        if frames.dim() == 3:
            frames = frames[..., None]
        kp, sc, ds, db, cnt = _native.ops().superpoint(frames.contiguous(), self._w, self.det_thr, self.max_kp,
                                                       self.nms_radius, self.border, bool(with_bf16))
        return kp, sc, ds, (db if with_bf16 else None), cnt

    def extract(self, images):
        """List of HxW[x3] uint8 numpy images (same size) -> list of dicts with numpy
        keypoints [n, 2], keypoint_scores [n], descriptors [n, 256]."""
        frames = torch.from_numpy(np.stack([np.asarray(im, np.uint8) for im in images])).to(self.device)
        kp, sc, ds, _, cnt = self.extract_device(frames)
        kp, sc, ds, cnt = kp.cpu().numpy(), sc.cpu().numpy(), ds.cpu().numpy(), cnt.cpu().numpy()
        return [{"keypoints": kp[i, :cnt[i]], "keypoint_scores": sc[i, :cnt[i]], "descriptors": ds[i, :cnt[i]]}
                for i in range(len(images))]
