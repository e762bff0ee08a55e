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
import functools
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


def superpoint_state_dict(seed=0, whiten=True):
    """Seeded float32 SuperPoint weights (He-normal convs, small biases), LightGlue key names.

    With ``whiten`` the descriptor head convDb (1x1, 256 -> 256) is set to the
    (regularised) whitening transform of convDa's responses on a few seeded synthetic
    scenes instead of random numbers.  Untrained ReLU features share one dominant
    direction (descriptor cosine ~0.9 between unrelated points), which leaves LightGlue
    nothing to match; whitened descriptors are decorrelated (cosine ~0 between
    unrelated points, > 0.95 between the same scene point in two views), so a revisit
    produces true correspondences -- the property a trained SuperPoint has."""
    return {k: v.copy() for k, v in _superpoint_sd(int(seed), bool(whiten)).items()}


@functools.lru_cache(maxsize=4)
def _superpoint_sd(seed, whiten):
    rng = np.random.default_rng(seed)
    sd = {}
    for name, cin, cout, k in SUPERPOINT_LAYERS:
        std = np.float32((2.0 / (cin * k * k)) ** 0.5)
        sd[f"{name}.weight"] = rng.standard_normal((cout, cin, k, k), dtype=np.float32) * std
        sd[f"{name}.bias"] = rng.standard_normal((cout,), dtype=np.float32) * np.float32(0.01)
    if whiten:
        sd["convDb.weight"], sd["convDb.bias"] = _whitening_head(sd, seed)
    return sd


def _whitening_head(sd, seed, n_scenes=4, reg=1e-2):
    """convDb = C^(-1/2) (eigenvalues floored at reg * max), bias = -C^(-1/2) mu, where mu / C
    are the mean / covariance of convDa's ReLU outputs over the descriptor grid of
    `n_scenes` seeded synthetic keyframes.  One-time weight construction on the CPU."""
    import torch
    import torch.nn.functional as F
    from . import synthetic
    imgs = []
    for i in range(n_scenes):
        base = synthetic.scene(50_000 + 97 * seed + i).astype(np.int16)
        noise = np.random.default_rng(seed * 131 + i).integers(0, 30, base.shape)
        imgs.append(np.clip(base + noise, 0, 255))
    bgr = np.stack(imgs).astype(np.int32)
    gray = ((bgr[..., 0] * 1868 + bgr[..., 1] * 9617 + bgr[..., 2] * 4899 + 8192) >> 14).astype(np.float32) / 255.0
    w = {k: torch.from_numpy(v) for k, v in sd.items()}
    with torch.no_grad():
        x = torch.from_numpy(gray)[:, None]
        for name in ("conv1a", "conv1b", "conv2a", "conv2b", "conv3a", "conv3b", "conv4a", "conv4b"):
            x = torch.relu(F.conv2d(x, w[name + ".weight"], w[name + ".bias"], padding=1))
            if name in ("conv1b", "conv2b", "conv3b"):
                x = F.max_pool2d(x, 2, 2)
        c = torch.relu(F.conv2d(x, w["convDa.weight"], w["convDa.bias"], padding=1))
    Z = c.permute(0, 2, 3, 1).reshape(-1, c.shape[1]).double().numpy()
    mu = Z.mean(0)
    ev, V = np.linalg.eigh(np.cov(Z.T))
    Wh = (V / np.sqrt(np.maximum(ev, 0) + reg * ev.max())) @ V.T
    return Wh.astype(np.float32).reshape(256, 256, 1, 1), (-(Wh @ mu)).astype(np.float32)


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


# ----------------------------------------------------------------- LightGlue
LG_DIM, LG_LAYERS = 256, 9


def lightglue_keys():
    keys = ["posenc.Wr.weight"]
    for i in range(LG_LAYERS):
        for blk, lins in (("self_attn", ("Wqkv", "out_proj")), ("cross_attn", ("to_qk", "to_v", "to_out"))):
            p = f"transformers.{i}.{blk}."
            for n in lins + ("ffn.0", "ffn.1", "ffn.3"):
                keys += [p + n + ".weight", p + n + ".bias"]
        keys += [f"log_assignment.{i}.matchability.weight", f"log_assignment.{i}.matchability.bias",
                 f"log_assignment.{i}.final_proj.weight", f"log_assignment.{i}.final_proj.bias"]
        if i < LG_LAYERS - 1:
            keys += [f"token_confidence.{i}.token.0.weight", f"token_confidence.{i}.token.0.bias"]
    return keys


def lightglue_state_dict(seed=0, res_gain=0.05, final_scale=16.0, match_gain=6.0, match_bias=3.0, conf_gain=6.0,
                         conf_bias=1.5):
    """Seeded float32 LightGlue(features='superpoint') weights with the package's key names.

    Untrained, but shaped so the network behaves like a matcher on SuperPoint-like
    inputs: small residual updates (``res_gain``) keep tokens close to their
    descriptors, final_proj ~ ``final_scale`` * I makes the assignment a sharpened
    descriptor similarity, and matchability / token-confidence spreads exercise point
    pruning and early stopping.
    """
    rng = np.random.default_rng(seed)
    d = LG_DIM

    def lin(o, i, gain=1.0):
        return (rng.standard_normal((o, i), dtype=np.float32) * np.float32(gain / np.sqrt(i)),
                rng.standard_normal((o,), dtype=np.float32) * np.float32(0.02))

    sd = {"posenc.Wr.weight": rng.standard_normal((32, 2), dtype=np.float32)}
    shapes = {"Wqkv": (3 * d, d), "out_proj": (d, d), "to_qk": (d, d), "to_v": (d, d), "to_out": (d, d),
              "ffn.0": (2 * d, 2 * d), "ffn.3": (d, 2 * d)}
    for i in range(LG_LAYERS):
        for blk, lins in (("self_attn", ("Wqkv", "out_proj")), ("cross_attn", ("to_qk", "to_v", "to_out"))):
            p = f"transformers.{i}.{blk}."
            for n in lins + ("ffn.0", "ffn.3"):
                w, b = lin(*shapes[n], gain=res_gain if n == "ffn.3" else 1.0)
                sd[p + n + ".weight"], sd[p + n + ".bias"] = w, b * np.float32(res_gain if n == "ffn.3" else 1.0)
            sd[p + "ffn.1.weight"] = 1.0 + rng.standard_normal(2 * d, dtype=np.float32) * np.float32(0.1)
            sd[p + "ffn.1.bias"] = rng.standard_normal(2 * d, dtype=np.float32) * np.float32(0.05)
        w, b = lin(1, d, gain=match_gain)
        sd[f"log_assignment.{i}.matchability.weight"] = w
        sd[f"log_assignment.{i}.matchability.bias"] = b + np.float32(match_bias)
        w, b = lin(d, d, gain=0.05)
        sd[f"log_assignment.{i}.final_proj.weight"] = w + np.eye(d, dtype=np.float32) * np.float32(final_scale)
        sd[f"log_assignment.{i}.final_proj.bias"] = b
        if i < LG_LAYERS - 1:
            w, b = lin(1, d, gain=conf_gain)
            sd[f"token_confidence.{i}.token.0.weight"] = w
            sd[f"token_confidence.{i}.token.0.bias"] = b + np.float32(conf_bias)
    return sd


def load_lightglue_state_dict(path):
    """LightGlue superpoint_lightglue.pth-style checkpoint from a local file (weights only)."""
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    import re
    # older releases stored "self_attn.{i}.*" / "cross_attn.{i}.*" (LightGlue renames them on load)
    sd = {re.sub(r"^(self_attn|cross_attn)\.(\d+)\.", r"transformers.\2.\1.", k.replace("matcher.", "")): v
          for k, v in sd.items()}
    missing = [k for k in lightglue_keys() if k not in sd]
    if missing:
        raise KeyError(f"checkpoint {path} lacks LightGlue keys, e.g. {missing[:3]}")
    return {k: sd[k].float().cpu().numpy() for k in lightglue_keys()}


def resolve_lightglue_state_dict(path=None, seed=0):
    path = path or os.environ.get("MLGATE_LIGHTGLUE_WEIGHTS")
    if path:
        return load_lightglue_state_dict(path), path
    return lightglue_state_dict(seed), f"synthetic(seed={seed})"


# ----------------------------------------------------------------- ResNet-50 (MixVPR / SALAD fallback)
RESNET_STAGES = ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))  # width, blocks, first stride


def resnet50_keys():
    keys = ["conv1.weight"] + [f"bn1.{s}" for s in ("weight", "bias", "running_mean", "running_var")]
    for li, (width, blocks, _) in enumerate(RESNET_STAGES, 1):
        for b in range(blocks):
            p = f"layer{li}.{b}."
            for c in (1, 2, 3):
                keys.append(p + f"conv{c}.weight")
                keys += [p + f"bn{c}.{s}" for s in ("weight", "bias", "running_mean", "running_var")]
            if b == 0:
                keys.append(p + "downsample.0.weight")
                keys += [p + f"downsample.1.{s}" for s in ("weight", "bias", "running_mean", "running_var")]
    return keys


def resnet50_state_dict(seed=0):
    """Seeded float32 torchvision resnet50 weights (He-normal convs, BatchNorm statistics
    around identity), torchvision key names, fc omitted (the fallback drops it)."""
    rng = np.random.default_rng(seed)
    sd = {}

    def conv(name, cout, cin, k, gain=1.0):
        std = np.float32(gain * np.sqrt(2.0 / (cin * k * k)))
        sd[name] = rng.standard_normal((cout, cin, k, k), dtype=np.float32) * std

    def bn(name, c, scale=1.0):
        sd[name + ".weight"] = (np.float32(scale) * (1.0 + 0.1 * rng.standard_normal(c))).astype(np.float32)
        sd[name + ".bias"] = (0.05 * rng.standard_normal(c)).astype(np.float32)
        sd[name + ".running_mean"] = (0.05 * rng.standard_normal(c)).astype(np.float32)
        sd[name + ".running_var"] = (1.0 + 0.2 * rng.random(c)).astype(np.float32)

    conv("conv1.weight", 64, 3, 7)
    bn("bn1", 64)
    cin = 64
    for li, (width, blocks, _) in enumerate(RESNET_STAGES, 1):
        for b in range(blocks):
            p = f"layer{li}.{b}."
            conv(p + "conv1.weight", width, cin, 1)
            bn(p + "bn1", width)
            conv(p + "conv2.weight", width, width, 3)
            bn(p + "bn2", width)
            conv(p + "conv3.weight", width * 4, width, 1)
            bn(p + "bn3", width * 4, scale=0.3)  # residual branch damped as in trained nets
            if b == 0:
                conv(p + "downsample.0.weight", width * 4, cin, 1)
                bn(p + "downsample.1", width * 4)
            cin = width * 4
    return sd


def load_resnet50_state_dict(path):
    """torchvision resnet50 checkpoint (e.g. resnet50-0676ba61.pth) from a local file."""
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    missing = [k for k in resnet50_keys() if k not in sd]
    if missing:
        raise KeyError(f"checkpoint {path} lacks resnet50 keys, e.g. {missing[:3]}")
    return {k: sd[k].float().cpu().numpy() for k in resnet50_keys()}


def resolve_resnet50_state_dict(path=None, seed=0):
    path = path or os.environ.get("MLGATE_RESNET50_WEIGHTS")
    if path:
        return load_resnet50_state_dict(path), path
    return resnet50_state_dict(seed), f"synthetic(seed={seed})"


# ----------------------------------------------------------------------------- LoFTR
# kornia.feature.LoFTR(pretrained='indoor') (geometric_verification.py:446-449): the
# ResNetFPN_8_2 backbone, the 8-layer coarse and 2-layer fine linear-attention
# transformers and the fine preprocessing, with kornia's state-dict key names.
LOFTR_DIMS = (128, 196, 256)


def loftr_keys():
    keys = ["backbone.conv1.weight"] + [f"backbone.bn1.{s}" for s in ("weight", "bias", "running_mean",
                                                                       "running_var")]
    bn = ("weight", "bias", "running_mean", "running_var")
    for li in range(3):
        for bi in range(2):
            p = f"backbone.layer{li + 1}.{bi}."
            keys += [p + "conv1.weight", p + "conv2.weight"] + [p + f"bn{j}.{s}" for j in (1, 2) for s in bn]
            if li > 0 and bi == 0:
                keys += [p + "downsample.0.weight"] + [p + f"downsample.1.{s}" for s in bn]
    keys += ["backbone.layer3_outconv.weight", "backbone.layer2_outconv.weight", "backbone.layer1_outconv.weight"]
    for n in (2, 1):
        p = f"backbone.layer{n}_outconv2."
        keys += [p + "0.weight", p + "3.weight"] + [p + f"1.{s}" for s in bn]
    for pre, nl in (("loftr_coarse", 8), ("loftr_fine", 2)):
        for i in range(nl):
            p = f"{pre}.layers.{i}."
            keys += [p + s for s in ("q_proj.weight", "k_proj.weight", "v_proj.weight", "merge.weight",
                                     "mlp.0.weight", "mlp.2.weight", "norm1.weight", "norm1.bias", "norm2.weight",
                                     "norm2.bias")]
    keys += ["fine_preprocess.down_proj.weight", "fine_preprocess.down_proj.bias",
             "fine_preprocess.merge_feat.weight", "fine_preprocess.merge_feat.bias"]
    return keys


def loftr_state_dict(seed=0, whiten=True):
    """Seeded float32 weights with kornia's LoFTR key names and shapes (He-normal convs,
    BatchNorm statistics near identity, 1 / sqrt(fan-in) linears; the transformers' norm2
    gains small, so each layer refines rather than replaces the token).

    With ``whiten`` the coarse lateral conv (layer3_outconv, 1x1 256 -> 256, no bias) is
    the regularised whitening of layer3's responses on a few seeded synthetic scenes, with
    their mean direction projected out: untrained ReLU features share one dominant
    direction, which leaves the dual-softmax nothing to match; whitened ones make a
    revisit produce confident coarse matches, as trained LoFTR features do."""
    return {k: v.copy() for k, v in _loftr_sd(int(seed), bool(whiten)).items()}


@functools.lru_cache(maxsize=2)
def _loftr_sd(seed, whiten):
    rng = np.random.default_rng(seed)
    sd = {}

    def normal(shape, std, mean=0.0):
        return (rng.standard_normal(shape, dtype=np.float32) * np.float32(std) + np.float32(mean)).astype(np.float32)

    def conv(name, cout, cin, k):
        sd[name] = normal((cout, cin, k, k), np.sqrt(2.0 / (cin * k * k)))

    def bn(p, c):
        sd[p + ".weight"] = rng.uniform(0.8, 1.2, c).astype(np.float32)
        sd[p + ".bias"] = normal((c,), 0.05)
        sd[p + ".running_mean"] = normal((c,), 0.1)
        sd[p + ".running_var"] = rng.uniform(0.6, 1.4, c).astype(np.float32)

    d0, d1, d2 = LOFTR_DIMS
    conv("backbone.conv1.weight", d0, 1, 7)
    bn("backbone.bn1", d0)
    cin = d0
    for li, d in enumerate(LOFTR_DIMS):
        for bi in range(2):
            p = f"backbone.layer{li + 1}.{bi}."
            conv(p + "conv1.weight", d, cin if bi == 0 else d, 3)
            conv(p + "conv2.weight", d, d, 3)
            bn(p + "bn1", d)
            bn(p + "bn2", d)
            if li > 0 and bi == 0:
                conv(p + "downsample.0.weight", d, cin, 1)
                bn(p + "downsample.1", d)
        cin = d
    conv("backbone.layer3_outconv.weight", d2, d2, 1)
    conv("backbone.layer2_outconv.weight", d2, d1, 1)
    conv("backbone.layer2_outconv2.0.weight", d2, d2, 3)
    bn("backbone.layer2_outconv2.1", d2)
    conv("backbone.layer2_outconv2.3.weight", d1, d2, 3)
    conv("backbone.layer1_outconv.weight", d1, d0, 1)
    conv("backbone.layer1_outconv2.0.weight", d1, d1, 3)
    bn("backbone.layer1_outconv2.1", d1)
    conv("backbone.layer1_outconv2.3.weight", d0, d1, 3)
    for pre, nl, d in (("loftr_coarse", 8, 256), ("loftr_fine", 2, 128)):
        for i in range(nl):
            p = f"{pre}.layers.{i}."
            for n in ("q_proj", "k_proj", "v_proj", "merge"):
                sd[p + n + ".weight"] = normal((d, d), 1.0 / np.sqrt(d))
            sd[p + "mlp.0.weight"] = normal((2 * d, 2 * d), np.sqrt(2.0 / (2 * d)))
            sd[p + "mlp.2.weight"] = normal((d, 2 * d), 1.0 / np.sqrt(2 * d))
            sd[p + "norm1.weight"] = normal((d,), 0.05, 1.0)
            sd[p + "norm1.bias"] = normal((d,), 0.02)
            sd[p + "norm2.weight"] = normal((d,), 0.02, 0.1)
            sd[p + "norm2.bias"] = normal((d,), 0.01)
    sd["fine_preprocess.down_proj.weight"] = normal((128, 256), 1.0 / 16)
    sd["fine_preprocess.down_proj.bias"] = normal((128,), 0.02)
    sd["fine_preprocess.merge_feat.weight"] = normal((128, 256), 1.0 / 16)
    sd["fine_preprocess.merge_feat.bias"] = normal((128,), 0.02)
    if whiten:
        sd["backbone.layer3_outconv.weight"] = _loftr_whitening(sd, seed)
    return sd


def _loftr_whitening(sd, seed, n_scenes=3, reg=1e-2, h=240, w=320):
    """Whitening of layer3's outputs (mean direction projected out) over the 1/8 grid of
    `n_scenes` seeded synthetic frames.  One-time weight construction on the CPU."""
    import torch
    import torch.nn.functional as F
    from . import synthetic
    t = {k: torch.from_numpy(v) for k, v in sd.items()}

    def bn(x, p):
        return F.batch_norm(x, t[p + ".running_mean"], t[p + ".running_var"], t[p + ".weight"], t[p + ".bias"],
                            False, 0.0, 1e-5)

    def block(x, p, stride):
        y = F.relu(bn(F.conv2d(x, t[p + ".conv1.weight"], stride=stride, padding=1), p + ".bn1"))
        y = bn(F.conv2d(y, t[p + ".conv2.weight"], padding=1), p + ".bn2")
        if stride != 1:
            x = bn(F.conv2d(x, t[p + ".downsample.0.weight"], stride=stride), p + ".downsample.1")
        return F.relu(x + y)

    imgs = []
    for i in range(n_scenes):
        base = synthetic.scene(70_000 + 97 * seed + i, h, w).astype(np.int32)
        imgs.append((base[..., 0] * 1868 + base[..., 1] * 9617 + base[..., 2] * 4899 + 8192) >> 14)
    with torch.no_grad():
        x = torch.from_numpy(np.stack(imgs).astype(np.float32) / 255.0)[:, None]
        x = F.relu(bn(F.conv2d(x, t["backbone.conv1.weight"], stride=2, padding=3), "backbone.bn1"))
        for li, stride in ((1, 1), (2, 2), (3, 2)):
            x = block(block(x, f"backbone.layer{li}.0", stride), f"backbone.layer{li}.1", 1)
    Z = x.permute(0, 2, 3, 1).reshape(-1, x.shape[1]).double().numpy()
    mu = Z.mean(0)
    P = np.eye(len(mu)) - np.outer(mu, mu) / (mu @ mu)
    Zp = Z @ P
    ev, V = np.linalg.eigh(np.cov(Zp.T))
    Wh = (V / np.sqrt(np.maximum(ev, 0) + reg * ev.max())) @ V.T @ P
    return Wh.astype(np.float32).reshape(len(mu), len(mu), 1, 1)


def load_loftr_state_dict(path):
    """kornia LoFTR checkpoint (loftr_indoor.ckpt: {'state_dict': ...} or a bare state dict)."""
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    sd = sd.get("state_dict", sd)
    missing = [k for k in loftr_keys() if k not in sd]
    if missing:
        raise KeyError(f"checkpoint {path} lacks LoFTR keys, e.g. {missing[:3]}")
    return {k: sd[k].float().cpu().numpy() for k in loftr_keys()}


def resolve_loftr_state_dict(path=None, seed=0):
    path = path or os.environ.get("MLGATE_LOFTR_WEIGHTS")
    if path:
        return load_loftr_state_dict(path), path
    return loftr_state_dict(seed), f"synthetic(seed={seed})"


# ----------------------------------------------------------------- SuperGlue (magicleap)
SG_DIM, SG_LAYERS = 256, 18
SG_KENC = (3, 32, 64, 128, 256, 256)  # KeypointEncoder MLP channels (layers [32, 64, 128, 256])


def superglue_keys():
    """magicleap superglue_{indoor,outdoor}.pth key names (eval: BatchNorm running stats)."""
    bn = ("weight", "bias", "running_mean", "running_var")
    keys = ["bin_score"]
    for i in range(len(SG_KENC) - 1):
        keys += [f"kenc.encoder.{3 * i}.weight", f"kenc.encoder.{3 * i}.bias"]
        if i < len(SG_KENC) - 2:
            keys += [f"kenc.encoder.{3 * i + 1}.{s}" for s in bn]
    for i in range(SG_LAYERS):
        p = f"gnn.layers.{i}."
        for n in ("attn.proj.0", "attn.proj.1", "attn.proj.2", "attn.merge", "mlp.0", "mlp.3"):
            keys += [p + n + ".weight", p + n + ".bias"]
        keys += [p + "mlp.1." + s for s in bn]
    return keys + ["final_proj.weight", "final_proj.bias"]


@functools.lru_cache(maxsize=2)
def superglue_state_dict(seed=0, res_gain=0.05, kenc_gain=0.05, final_scale=12.0, bin_score=1.0):
    """Seeded float32 SuperGlue weights with magicleap's key names and Conv1d shapes.

    Untrained but matcher-like on SuperPoint descriptors: small residual GNN updates
    (``res_gain``) and a small keypoint encoding (``kenc_gain``) keep the states near the
    unit descriptors, final_proj ~ ``final_scale`` * I turns the Sinkhorn input into a
    sharpened descriptor similarity (scores / 16 ~ 9 cos), and eval BatchNorms with
    non-trivial running statistics exercise the folding.
    """
    rng = np.random.default_rng(seed + 7000)
    f = np.float32

    def conv(o, i, gain=1.0):
        return (rng.standard_normal((o, i, 1), dtype=f) * f(gain / np.sqrt(i)),
                rng.standard_normal((o,), dtype=f) * f(0.02 * gain))

    def bn(p, c):
        return {p + "weight": f(1.0) + rng.standard_normal(c, dtype=f) * f(0.1),
                p + "bias": rng.standard_normal(c, dtype=f) * f(0.05),
                p + "running_mean": rng.standard_normal(c, dtype=f) * f(0.05),
                p + "running_var": rng.uniform(0.5, 1.5, c).astype(f)}

    sd = {"bin_score": np.array(bin_score, f)}
    n = len(SG_KENC) - 1
    for i in range(n):
        last = i == n - 1
        w, b = conv(SG_KENC[i + 1], SG_KENC[i], kenc_gain if last else 1.0)
        sd[f"kenc.encoder.{3 * i}.weight"], sd[f"kenc.encoder.{3 * i}.bias"] = w, b
        if not last:
            sd.update(bn(f"kenc.encoder.{3 * i + 1}.", SG_KENC[i + 1]))
    d = SG_DIM
    for i in range(SG_LAYERS):
        p = f"gnn.layers.{i}."
        for k in range(3):
            sd[p + f"attn.proj.{k}.weight"], sd[p + f"attn.proj.{k}.bias"] = conv(d, d)
        sd[p + "attn.merge.weight"], sd[p + "attn.merge.bias"] = conv(d, d)
        sd[p + "mlp.0.weight"], sd[p + "mlp.0.bias"] = conv(2 * d, 2 * d)
        sd.update(bn(p + "mlp.1.", 2 * d))
        w, _ = conv(d, 2 * d, res_gain)
        sd[p + "mlp.3.weight"], sd[p + "mlp.3.bias"] = w, np.zeros(d, f)  # constant_(bias, 0.0) as upstream
    w, b = conv(d, d, 0.05)
    sd["final_proj.weight"] = w + (np.eye(d, dtype=f) * f(final_scale))[:, :, None]
    sd["final_proj.bias"] = b
    return sd


def load_superglue_state_dict(path):
    """magicleap superglue_*.pth from a local file (weights only)."""
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    missing = [k for k in superglue_keys() if k not in sd]
    if missing:
        raise KeyError(f"checkpoint {path} lacks SuperGlue keys, e.g. {missing[:3]}")
    return {k: sd[k].float().cpu().numpy() for k in superglue_keys()}


def resolve_superglue_state_dict(path=None, seed=0):
    path = path or os.environ.get("MLGATE_SUPERGLUE_WEIGHTS")
    if path:
        return load_superglue_state_dict(path), path
    return superglue_state_dict(seed), f"synthetic(seed={seed})"


# ----------------------------------------------------------------- SALAD
# serizba/salad VPRModel state dict (SALAD, place_recognition.py:357-368): the hub
# DINOv2 backbone under ``backbone.model.`` and the SALAD aggregator (num_channels 768,
# num_clusters 64, cluster_dim 128, token_dim 256).
SALAD_CLUSTERS, SALAD_CLUSTER_DIM, SALAD_TOKEN_DIM = 64, 128, 256


def salad_aggregator_shapes():
    c = EMBED
    return {"token_features.0.weight": (512, c), "token_features.0.bias": (512,),
            "token_features.2.weight": (SALAD_TOKEN_DIM, 512), "token_features.2.bias": (SALAD_TOKEN_DIM,),
            "cluster_features.0.weight": (512, c, 1, 1), "cluster_features.0.bias": (512,),
            "cluster_features.3.weight": (SALAD_CLUSTER_DIM, 512, 1, 1),
            "cluster_features.3.bias": (SALAD_CLUSTER_DIM,),
            "score.0.weight": (512, c, 1, 1), "score.0.bias": (512,),
            "score.3.weight": (SALAD_CLUSTERS, 512, 1, 1), "score.3.bias": (SALAD_CLUSTERS,),
            "dust_bin": ()}


def salad_keys():
    return ["backbone.model." + k for k in hub_keys()] + ["aggregator." + k for k in salad_aggregator_shapes()]


def salad_state_dict(seed=0, score_gain=2.0):
    """Seeded float32 weights with serizba/salad's key names and shapes (He-normal hidden
    layers; ``score_gain`` widens the cluster scores so the Sinkhorn plan is not flat)."""
    sd = {"backbone.model." + k: v for k, v in synthetic_state_dict(seed).items()}
    rng = np.random.default_rng(seed + 7)
    for k, shp in salad_aggregator_shapes().items():
        if k == "dust_bin":
            sd["aggregator.dust_bin"] = np.float32(1.0).reshape(())
            continue
        if k.endswith("bias"):
            sd["aggregator." + k] = (rng.standard_normal(shp, dtype=np.float32) * np.float32(0.02))
            continue
        fan_in = int(np.prod(shp[1:]))
        std = np.sqrt(2.0 / fan_in) if k.split(".")[1] == "0" else np.sqrt(1.0 / fan_in)
        if k.startswith("score.3"):
            std *= score_gain
        sd["aggregator." + k] = rng.standard_normal(shp, dtype=np.float32) * np.float32(std)
    return sd


def load_salad_state_dict(path):
    """serizba/salad checkpoint (VPRModel state dict, optionally under 'state_dict') from a
    local file, weights only."""
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    missing = [k for k in salad_keys() if k not in sd]
    if missing:
        raise KeyError(f"checkpoint {path} lacks SALAD keys, e.g. {missing[:3]}")
    return {k: sd[k].float().cpu().numpy() for k in salad_keys()}


def resolve_salad_state_dict(path=None, seed=0):
    path = path or os.environ.get("MLGATE_SALAD_WEIGHTS")
    if path:
        return load_salad_state_dict(path), path
    return salad_state_dict(seed), f"synthetic(seed={seed})"
