"""DINOv2 ViT-B/14 weights for the CricaVPR descriptor path.

The reference fetches ``torch.hub.load('facebookresearch/dinov2', 'dinov2_vitb14')``
(place_recognition.py:586-590).  There is no network here or on the GPU box, so:

  * ``load_hub_state_dict(path)`` reads a hub-format checkpoint from a local path with
    ``torch.load(weights_only=True)`` (``pretrained_path`` / ``MLGATE_DINOV2_WEIGHTS``);
  * otherwise ``synthetic_state_dict(seed)`` builds seeded random weights of exactly
    the hub architecture and key names, so the full network runs with real shapes.
    Descriptors from synthetic weights are meaningful for throughput and parity
    testing only, not for place recognition.
"""
import os

import numpy as np

EMBED, DEPTH, HEADS, MLP, PATCH, POS_GRID = 768, 12, 12, 3072, 14, 37


def hub_keys():
    keys = ["cls_token", "pos_embed", "patch_embed.proj.weight", "patch_embed.proj.bias",
            "norm.weight", "norm.bias"]
    for i in range(DEPTH):
        p = f"blocks.{i}."
        keys += [p + s for s in ("norm1.weight", "norm1.bias", "attn.qkv.weight", "attn.qkv.bias",
                                 "attn.proj.weight", "attn.proj.bias", "ls1.gamma", "norm2.weight",
                                 "norm2.bias", "mlp.fc1.weight", "mlp.fc1.bias", "mlp.fc2.weight",
                                 "mlp.fc2.bias", "ls2.gamma")]
    return keys


def synthetic_state_dict(seed=0):
    """Seeded float32 weights with the hub dinov2_vitb14 key names and shapes."""
    rng = np.random.default_rng(seed)

    def normal(shape, std, mean=0.0):
        a = rng.standard_normal(shape, dtype=np.float32) * np.float32(std)
        return a + np.float32(mean) if mean else a

    sd = {
        "cls_token": normal((1, 1, EMBED), 0.02),
        "pos_embed": normal((1, 1 + POS_GRID * POS_GRID, EMBED), 0.02),
        "patch_embed.proj.weight": normal((EMBED, 3, PATCH, PATCH), 0.02),
        "patch_embed.proj.bias": normal((EMBED,), 0.02),
        "norm.weight": normal((EMBED,), 0.1, 1.0),
        "norm.bias": normal((EMBED,), 0.05),
    }
    for i in range(DEPTH):
        p = f"blocks.{i}."
        sd[p + "norm1.weight"] = normal((EMBED,), 0.1, 1.0)
        sd[p + "norm1.bias"] = normal((EMBED,), 0.05)
        sd[p + "attn.qkv.weight"] = normal((3 * EMBED, EMBED), 0.05)
        sd[p + "attn.qkv.bias"] = normal((3 * EMBED,), 0.02)
        sd[p + "attn.proj.weight"] = normal((EMBED, EMBED), 0.03)
        sd[p + "attn.proj.bias"] = normal((EMBED,), 0.02)
        sd[p + "ls1.gamma"] = rng.uniform(0.05, 0.6, EMBED).astype(np.float32)
        sd[p + "norm2.weight"] = normal((EMBED,), 0.1, 1.0)
        sd[p + "norm2.bias"] = normal((EMBED,), 0.05)
        sd[p + "mlp.fc1.weight"] = normal((MLP, EMBED), 0.03)
        sd[p + "mlp.fc1.bias"] = normal((MLP,), 0.02)
        sd[p + "mlp.fc2.weight"] = normal((EMBED, MLP), 0.02)
        sd[p + "mlp.fc2.bias"] = normal((EMBED,), 0.02)
        sd[p + "ls2.gamma"] = rng.uniform(0.05, 0.6, EMBED).astype(np.float32)
    return sd


def load_hub_state_dict(path):
    """Hub-format dinov2_vitb14 checkpoint from a local file (no code executed from it)."""
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if "model" in sd and isinstance(sd["model"], dict):
        sd = sd["model"]
    missing = [k for k in hub_keys() if k not in sd]
    if missing:
        raise KeyError(f"checkpoint {path} lacks dinov2_vitb14 keys, e.g. {missing[:3]}")
    return {k: sd[k].float().cpu().numpy() for k in hub_keys()}


def resolve_state_dict(pretrained_path=None, seed=0):
    """(state_dict, source) -- local checkpoint if given/configured, else synthetic."""
    path = pretrained_path or os.environ.get("MLGATE_DINOV2_WEIGHTS")
    if path:
        return load_hub_state_dict(path), path
    return synthetic_state_dict(seed), f"synthetic(seed={seed})"


# ----------------------------------------------------------------- SuperPoint
# LightGlue's SuperPoint (geometric_verification.py:224-233): layer name, Cin, Cout, kernel
SUPERPOINT_LAYERS = [("conv1a", 1, 64, 3), ("conv1b", 64, 64, 3), ("conv2a", 64, 64, 3), ("conv2b", 64, 64, 3),
                     ("conv3a", 64, 128, 3), ("conv3b", 128, 128, 3), ("conv4a", 128, 128, 3),
                     ("conv4b", 128, 128, 3), ("convPa", 128, 256, 3), ("convPb", 256, 65, 1),
                     ("convDa", 128, 256, 3), ("convDb", 256, 256, 1)]


def superpoint_state_dict(seed=0):
    """Seeded float32 SuperPoint weights (He-normal convs, small biases), LightGlue key names."""
    rng = np.random.default_rng(seed)
    sd = {}
    for name, cin, cout, k in SUPERPOINT_LAYERS:
        std = np.float32((2.0 / (cin * k * k)) ** 0.5)
        sd[f"{name}.weight"] = rng.standard_normal((cout, cin, k, k), dtype=np.float32) * std
        sd[f"{name}.bias"] = rng.standard_normal((cout,), dtype=np.float32) * np.float32(0.01)
    return sd


def load_superpoint_state_dict(path):
    """LightGlue superpoint_v1.pth-style checkpoint from a local file (weights only)."""
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    keys = [f"{n}.{p}" for n, *_ in SUPERPOINT_LAYERS for p in ("weight", "bias")]
    missing = [k for k in keys if k not in sd]
    if missing:
        raise KeyError(f"checkpoint {path} lacks SuperPoint keys, e.g. {missing[:3]}")
    return {k: sd[k].float().cpu().numpy() for k in keys}


def resolve_superpoint_state_dict(path=None, seed=0):
    path = path or os.environ.get("MLGATE_SUPERPOINT_WEIGHTS")
    if path:
        return load_superpoint_state_dict(path), path
    return superpoint_state_dict(seed), f"synthetic(seed={seed})"
