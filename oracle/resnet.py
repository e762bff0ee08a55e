"""Oracle for the MixVPR / SALAD ResNet-50 fallback descriptor (test infrastructure only).

What the reference executes for MixVPR, SALAD and every DINOv2 failure is
``MixVPR._load_fallback_model`` + ``extract_descriptor``
(scripts/semantic_gating/place_recognition.py:248-306):
  transforms.ToPILImage() (the BGR array taken as RGB, no swap) -> Resize((224, 224))
  (Pillow bilinear, antialiased) -> ToTensor (/255) -> Normalize(ImageNet mean / std)
  -> torchvision resnet50 without fc (global average pool) -> 2048 floats, zero-padded
  to descriptor_dim (truncated if larger).
torchvision and the ImageNet weights are absent here; the network is restated in
torch-fp32 (eval-mode BatchNorm) and run with seeded synthetic weights (the product's
generator, mlgate.weights.resnet50_state_dict), pinned architecturally against
``transformers.ResNetModel``; the resize is restated from Pillow's Resample.c
(PRECISION_BITS = 22 fixed point, horizontal pass then vertical, uint8 in between)
and pinned bit-exact against Pillow itself (installed here).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

PRECISION_BITS = 22
MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)
STAGES = ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))  # width, blocks, stride


def bilinear_coeffs(in_size, out_size):
    """Pillow precompute_coeffs + normalize_coeffs_8bpc for the bilinear filter:
    (xmin [out], xmax [out], int32 kk [out, ksize])."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    xmins = np.zeros(out_size, np.int64)
    xmaxs = np.zeros(out_size, np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        ww = 0.0
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            v = 1.0 - t if t < 1.0 else 0.0
            w.append(v)
            ww += v
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + k * (1 << PRECISION_BITS)) if k < 0 else int(0.5 + k * (1 << PRECISION_BITS))
        xmins[xx], xmaxs[xx] = xmin, xmax
    return xmins, xmaxs, kk


def _pass(img, axis, out_size):
    """One Pillow 8bpc resample pass along axis (1 = horizontal, 0 = vertical)."""
    xmins, xmaxs, kk = bilinear_coeffs(img.shape[axis], out_size)
    src = np.moveaxis(img.astype(np.int64), axis, 0)
    out = np.empty((out_size,) + src.shape[1:], np.int64)
    for o in range(out_size):
        seg = src[xmins[o]:xmins[o] + xmaxs[o]]
        acc = (1 << (PRECISION_BITS - 1)) + np.tensordot(kk[o, :xmaxs[o]], seg, axes=(0, 0))
        out[o] = np.clip(acc >> PRECISION_BITS, 0, 255)
    return np.moveaxis(out, 0, axis).astype(np.uint8)


def pil_resize_bilinear(img, size):
    """Image.fromarray(img).resize((w, h), BILINEAR) for uint8 HxWx3 / HxW."""
    h, w = size
    out = img
    if w != img.shape[1]:
        out = _pass(out, 1, w)
    if h != img.shape[0]:
        out = _pass(out, 0, h)
    return out


def preprocess(image):
    """The fallback transform (place_recognition.py:262-270, 282-287) -> float32 [3, 224, 224]."""
    img = np.asarray(image)
    if img.ndim == 2:
        img = np.stack([img] * 3, axis=-1)
    elif img.shape[2] == 4:
        img = img[:, :, :3]
    r = pil_resize_bilinear(img.astype(np.uint8), (224, 224))
    t = torch.from_numpy(r).permute(2, 0, 1).float().div(255)
    mean = torch.tensor(MEAN).view(3, 1, 1)
    std = torch.tensor(STD).view(3, 1, 1)
    return (t - mean) / std


def _bn(x, sd, p):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        training=False, eps=1e-5)


def resnet50_features(sd, x):
    """torchvision resnet50 children()[:-1] on x [B, 3, H, W] -> [B, 2048, 1, 1]."""
    sd = {k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in sd.items()}
    x = F.relu(_bn(F.conv2d(x, sd["conv1.weight"], stride=2, padding=3), sd, "bn1"))
    x = F.max_pool2d(x, 3, 2, 1)
    for li, (width, blocks, stride) in enumerate(STAGES, 1):
        for b in range(blocks):
            p = f"layer{li}.{b}"
            s = stride if b == 0 else 1
            idt = x
            y = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"]), sd, p + ".bn1"))
            y = F.relu(_bn(F.conv2d(y, sd[p + ".conv2.weight"], stride=s, padding=1), sd, p + ".bn2"))
            y = _bn(F.conv2d(y, sd[p + ".conv3.weight"]), sd, p + ".bn3")
            if b == 0:
                idt = _bn(F.conv2d(x, sd[p + ".downsample.0.weight"], stride=s), sd, p + ".downsample.1")
            x = F.relu(y + idt)
    return F.adaptive_avg_pool2d(x, 1)


def extract_descriptor(sd, image, descriptor_dim=4096):
    """MixVPR.extract_descriptor on the fallback path -> float32 [descriptor_dim]."""
    with torch.no_grad():
        d = resnet50_features(sd, preprocess(image)[None]).numpy().flatten()
    if len(d) > descriptor_dim:
        return d[:descriptor_dim]
    return np.pad(d, (0, descriptor_dim - len(d)))
