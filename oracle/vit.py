"""Oracle for the CricaVPR descriptor path (test infrastructure only).

What the reference actually executes for vpr_method='cricavpr' (SURVEY.md §8a a1-a4):

  a1  CricaVPR._preprocess (place_recognition.py:781-803): cv2.resize to 322x322
      INTER_LINEAR (restated in oracle.c, parity unpinned vs OpenCV), gray/BGRA/BGR
      -> RGB, float32 / 255, (x - mean) / std with float64 ImageNet constants,
      -> float32 [1, 3, 322, 322].
  a2  torch.hub dinov2_vitb14 .get_intermediate_layers(x, n=1)[0] (:634):
      patch-embed conv 14/14, CLS token, pos-embed 37x37 bicubic-resampled with
      scale_factor (23 + 0.1) / 37 (antialias off), 12 pre-LN blocks (LN eps 1e-6,
      12 heads x 64, qkv bias, LayerScale, MLP 3072 exact-erf GELU), final LN,
      CLS stripped -> [B, 529, 768].
  a3  GeM (:636-641): drop patch token 0, clamp(min=1e-6)^3, mean over tokens, ^(1/3).
  a4  extract_local_features (:645-667): the same forward's features[:, 1:, :].

The network is restated in float32 torch ops on the CPU from the published hub
architecture; tests pin it against transformers.Dinov2Model (the same network) with
seeded weights.  Weights are a hub-format state_dict of numpy/torch arrays.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib

MEAN = np.array([0.485, 0.456, 0.406])
STD = np.array([0.229, 0.224, 0.225])
EMBED, HEADS, DEPTH, PATCH = 768, 12, 12, 14


def preprocess(image, size=322, swap_rb=True):
    """uint8 HxW / HxWx3 (BGR) / HxWx4 (BGRA) -> float32 [1, 3, size, size].

    swap_rb=False is AnyLoc._preprocess (place_recognition.py:489-505), which only
    converts gray and feeds 3-channel frames in stored (BGR) order."""
    img = np.asarray(image, dtype=np.uint8)
    r = _lib.resize_linear_u8(img, size, size)
    if r.ndim == 2:
        rgb = np.stack([r, r, r], axis=-1)
    elif not swap_rb:
        rgb = r[:, :, :3]
    elif r.shape[2] == 4:
        rgb = r[:, :, [2, 1, 0]]
    else:
        rgb = r[:, :, ::-1]
    x = rgb.astype(np.float32) / 255.0
    x = (x - MEAN) / STD
    return torch.from_numpy(np.ascontiguousarray(x)).permute(2, 0, 1).unsqueeze(0).float()


def _t(sd, k):
    v = sd[k]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))


def interpolate_pos_embed(pos_embed, grid):
    """Hub DinoVisionTransformer.interpolate_pos_encoding for a square grid."""
    pos_embed = pos_embed.float()
    n = pos_embed.shape[1] - 1
    m = int(math.sqrt(n))
    if grid == m:
        return pos_embed
    s = float(grid + 0.1) / m
    patch = pos_embed[:, 1:].reshape(1, m, m, -1).permute(0, 3, 1, 2)
    patch = F.interpolate(patch, mode="bicubic", antialias=False, scale_factor=(s, s))
    assert patch.shape[-2:] == (grid, grid)
    patch = patch.permute(0, 2, 3, 1).reshape(1, grid * grid, -1)
    return torch.cat((pos_embed[:, :1], patch), dim=1)


@torch.no_grad()
def forward_tokens(x, sd):
    """get_intermediate_layers(x, n=1, norm=True)[0]: [B, 3, S, S] -> [B, (S/14)^2, 768]."""
    return forward_tokens_with_cls(x, sd)[:, 1:]


@torch.no_grad()
def forward_tokens_with_cls(x, sd):
    """The hub forward through the final LayerNorm, CLS kept: [B, 1 + (S/14)^2, 768]
    (SALAD's DINOv2 backbone with norm_layer / return_token)."""
    B, _, S, _ = x.shape
    grid = S // PATCH
    t = F.conv2d(x, _t(sd, "patch_embed.proj.weight"), _t(sd, "patch_embed.proj.bias"), stride=PATCH)
    t = t.flatten(2).transpose(1, 2)
    cls = _t(sd, "cls_token").expand(B, -1, -1)
    t = torch.cat((cls, t), dim=1)
    t = t + interpolate_pos_embed(_t(sd, "pos_embed"), grid)
    T = t.shape[1]
    hd = EMBED // HEADS
    for i in range(DEPTH):
        p = f"blocks.{i}."
        h = F.layer_norm(t, (EMBED,), _t(sd, p + "norm1.weight"), _t(sd, p + "norm1.bias"), eps=1e-6)
        qkv = F.linear(h, _t(sd, p + "attn.qkv.weight"), _t(sd, p + "attn.qkv.bias"))
        qkv = qkv.reshape(B, T, 3, HEADS, hd).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0] * hd ** -0.5, qkv[1], qkv[2]
        a = (q @ k.transpose(-2, -1)).softmax(dim=-1)
        o = (a @ v).transpose(1, 2).reshape(B, T, EMBED)
        o = F.linear(o, _t(sd, p + "attn.proj.weight"), _t(sd, p + "attn.proj.bias"))
        t = t + o * _t(sd, p + "ls1.gamma")
        h = F.layer_norm(t, (EMBED,), _t(sd, p + "norm2.weight"), _t(sd, p + "norm2.bias"), eps=1e-6)
        h = F.gelu(F.linear(h, _t(sd, p + "mlp.fc1.weight"), _t(sd, p + "mlp.fc1.bias")))
        h = F.linear(h, _t(sd, p + "mlp.fc2.weight"), _t(sd, p + "mlp.fc2.bias"))
        t = t + h * _t(sd, p + "ls2.gamma")
    return F.layer_norm(t, (EMBED,), _t(sd, "norm.weight"), _t(sd, "norm.bias"), eps=1e-6)


def gem(features, p=3.0):
    """place_recognition.py:636-641 on get_intermediate_layers output."""
    patch = features[:, 1:, :]
    return patch.clamp(min=1e-6).pow(p).mean(dim=1).pow(1.0 / p)


@torch.no_grad()
def extract_descriptor(image, sd):
    """CricaVPR.extract_descriptor (DINOv2 + GeM path) -> float32 (768,)."""
    return gem(forward_tokens(preprocess(image), sd)).cpu().numpy().flatten()


@torch.no_grad()
def extract_local_features(image, sd):
    """CricaVPR.extract_local_features -> float32 [1, 528, 768]."""
    return forward_tokens(preprocess(image), sd)[:, 1:, :].cpu().numpy()


@torch.no_grad()
def anyloc_descriptor(image, sd):
    """AnyLoc.extract_descriptor (place_recognition.py:467-487): 518^2, patch mean -> (768,)."""
    f = forward_tokens(preprocess(image, 518, swap_rb=False), sd)
    return f[:, 1:, :].mean(dim=1).cpu().numpy().flatten()
