"""DINOv2 ViT-B/14 + GeM descriptor engine (CricaVPR path) on the mlgate HIP kernels.

Device-resident replacement for what CricaVPR does per keyframe
(place_recognition.py:613-667, 759-803): preprocessing, the hub
``get_intermediate_layers`` forward, GeM pooling and the local-feature cache -- all
from ONE forward (the reference runs the identical forward twice per add_image, once
for the descriptor and once for the local features).  Frames go in as uint8
[B, H, W, C] device tensors; everything up to the float32 descriptors stays in HBM.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import _native
from .weights import DEPTH, EMBED, PATCH

PATCH_K = 768  # 3*14*14 = 588 patch inputs zero-padded to 12 K-tiles of 64 (include/mlgate.h)
BLOCK_ORDER = ("norm1_w", "norm1_b", "qkv_w", "qkv_b", "proj_w", "proj_b", "ls1", "norm2_w", "norm2_b", "fc1_w",
               "fc1_b", "fc2_w", "fc2_b", "ls2")  # mlg_vit_block field order
BF16_FIELDS = {"qkv_w", "proj_w", "fc1_w", "fc2_w"}  # GEMM weights; everything else float32


def resample_pos_embed(pos_embed, grid):
    """Hub DinoVisionTransformer.interpolate_pos_encoding (square input): bicubic,
    scale_factor (grid + 0.1) / 37, antialias off.  One-time weight transform."""
    pos_embed = pos_embed.float()
    m = int(math.sqrt(pos_embed.shape[1] - 1))
    if grid == m:
        return pos_embed
    s = float(grid + 0.1) / m
    patch = pos_embed[:, 1:].reshape(1, m, m, -1).permute(0, 3, 1, 2)
    patch = F.interpolate(patch, mode="bicubic", antialias=False, scale_factor=(s, s))
    patch = patch.permute(0, 2, 3, 1).reshape(1, grid * grid, -1)
    return torch.cat((pos_embed[:, :1], patch), dim=1).contiguous()


MLG_VIT_SPLIT = 4  # include/mlgate.h


def split_weight(w):
    """[out, in] float32 -> bf16 [out, 2 in] = [W_hi | W_lo] (MLG_VIT_SPLIT packing:
    hi = bf16(W), lo = bf16(W - hi), so W = hi + lo to 2^-17)."""
    w = w.to(torch.float32)
    hi = w.to(torch.bfloat16)
    lo = (w - hi.to(torch.float32)).to(torch.bfloat16)
    return torch.cat([hi, lo], dim=1).contiguous()


class VitB14:
    """Packed device weights + workspace for batched CricaVPR descriptor extraction.

    precise=True selects the split-bf16 forward (MLG_VIT_SPLIT, include/mlgate.h): every
    GEMM and attention operand carried as a hi + lo bf16 pair, three MFMA products each.
    Descriptors then agree with the fp32 network to ~1e-11 (1 - cos) instead of ~1e-5, and
    kNN rankings over near-identical descriptors follow the fp32 reference's
    (tests/test_bench_parity_gpu.py).  It is the default everywhere the descriptors feed
    retrieval (DeviceGate, the CricaVPR / AnyLoc drop-ins); precise=False keeps the plain
    bf16 forward (3x fewer MFMA products; SALAD's trunk, A/B tools)."""

    def __init__(self, state_dict, device="cuda", image_size=322, max_batch=64, pool="gem", swap_rb=True,
                 precise=True):
        self.device = _native.require_device(device)
        if image_size % PATCH:
            raise ValueError("image_size must be a multiple of 14")
        self.image_size, self.grid = image_size, image_size // PATCH
        self.n_patches = self.grid * self.grid
        self.n_local = self.n_patches - 1  # tokens 2.. of get_intermediate_layers (CLS + patch 0 dropped)
        self.max_batch = max_batch
        self.precise = bool(precise)
        self.flags = ((1 if pool == "mean" else 0) | (0 if swap_rb else 2)  # MLG_VIT_POOL_MEAN / KEEP_CHANNELS
                      | (MLG_VIT_SPLIT if self.precise else 0))
        self._w = self._pack(state_dict)

    # ------------------------------------------------------------ weights
    def _dev(self, a, dtype):
        t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
        return t.to(self.device, torch.float32).to(dtype).contiguous()

    def _pack(self, sd):
        """Device tensors in mlg_vit_weights order (torch.ops.mlgate.vit_forward_into)."""
        f32, bf = torch.float32, torch.bfloat16
        pw = torch.as_tensor(np.asarray(sd["patch_embed.proj.weight"], np.float32)).reshape(EMBED, -1)
        pos = torch.as_tensor(np.asarray(sd["pos_embed"], np.float32)).to(self.device)

        def gemm_w(a):  # a GEMM weight in the layout of this forward
            t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
            t = t.to(self.device, torch.float32)
            return split_weight(t) if self.precise else t.to(bf).contiguous()
        w = [gemm_w(F.pad(pw, (0, PATCH_K - pw.shape[1]))), self._dev(sd["patch_embed.proj.bias"], f32),
             self._dev(np.asarray(sd["cls_token"], np.float32).reshape(EMBED), f32),
             self._dev(resample_pos_embed(pos, self.grid).reshape(-1, EMBED), f32)]
        names = {"norm1_w": "norm1.weight", "norm1_b": "norm1.bias", "qkv_w": "attn.qkv.weight",
                 "qkv_b": "attn.qkv.bias", "proj_w": "attn.proj.weight", "proj_b": "attn.proj.bias",
                 "ls1": "ls1.gamma", "norm2_w": "norm2.weight", "norm2_b": "norm2.bias", "fc1_w": "mlp.fc1.weight",
                 "fc1_b": "mlp.fc1.bias", "fc2_w": "mlp.fc2.weight", "fc2_b": "mlp.fc2.bias", "ls2": "ls2.gamma"}
        for i in range(DEPTH):
            for f in BLOCK_ORDER:
                v = sd[f"blocks.{i}." + names[f]]
                w.append(gemm_w(v) if f in BF16_FIELDS else self._dev(v, f32))
        w += [self._dev(sd["norm.weight"], f32), self._dev(sd["norm.bias"], f32)]
        return w

    # ------------------------------------------------------------ forward
    def forward_into(self, frames, desc_out, local_out=None):
        """frames: uint8 [B, H, W, C] device tensor (C = 1, 3 BGR or 4 BGRA; or [B, H, W]).
        Writes float32 descriptors [B, 768] (and local features [B, n_local, 768]);
        torch.ops.mlgate.vit_forward_into on the current stream."""
        if frames.dim() == 3:
            frames = frames.unsqueeze(-1)
        if frames.dtype != torch.uint8 or frames.device.type != "cuda":
            raise TypeError("frames must be a uint8 tensor on the HIP device")
        _native.ops().vit_forward_into(frames.contiguous(), self._w, self.image_size, self.flags, self.max_batch,
                                       desc_out, local_out)

    def forward(self, frames, with_local=False):
        B = frames.shape[0]
        desc = torch.empty(B, EMBED, dtype=torch.float32, device=self.device)
        local = (torch.empty(B, self.n_local, EMBED, dtype=torch.float32, device=self.device)
                 if with_local else None)
        self.forward_into(frames, desc, local)
        return (desc, local) if with_local else desc
