"""Oracle for the SuperPoint keypoint detector / descriptor (test infrastructure only).

The reference calls LightGlue's SuperPoint (geometric_verification.py:224-233,
263-312: ``SuperPoint(max_num_keypoints=2048, detection_threshold=0.001)`` on
``cv2.cvtColor(img, COLOR_BGR2GRAY) / 255``).  That package (github cvg/LightGlue,
unpinned HEAD) and its trained weights are absent here, so this is a torch-fp32 CPU
restatement of its published forward pass, run with the same seeded synthetic
weights as the GPU path; parity is against this restatement ("unpinned" w.r.t. the
trained model).  Semantics restated:
  * cv2 BGR2GRAY for 8-bit: (1868 B + 9617 G + 4899 R + 8192) >> 14;
  * VGG encoder conv1a..conv4b (3x3, ReLU), 2x2 max-pool after conv1b/2b/3b;
  * detector head convPa (3x3, ReLU) -> convPb (1x1, 65) -> softmax over 65 channels,
    dustbin dropped, 8x8 depth-to-space;
  * simple_nms (radius 4): max-pool 9x9 equality mask + two suppression rounds;
  * borders of 4 px set to -1, keep scores > detection_threshold (torch.where order =
    raster), top-k (k = 2048) by score, sorted, only when there are more than k;
  * descriptor head convDa (3x3, ReLU) -> convDb (1x1, 256) -> L2 normalise ->
    bilinear grid_sample (align_corners=True) at (kp - s/2 + 0.5) / (size*s - s/2 - 0.5)
    -> L2 normalise.
Weights come from the caller (the product's seeded generator,
mlgate.weights.superpoint_state_dict, or a checkpoint).  ``emulate_bf16`` rounds weights and every stored activation to bfloat16 the way the
GPU kernels store them, so GPU-vs-oracle differences reduce to summation order.
Precision probes (tools/lg_precision_probe.py) split it: ``sites`` = {'w'} rounds only the
weights, {'act'} only the stored activations; ``tf32`` rounds every conv's input and
weights to TF32 (10-bit mantissa, round to nearest) -- what cuDNN does by default on
Ampere and later NVIDIA GPUs (torch.backends.cudnn.allow_tf32 defaults to True), the
reference's SuperPoint on CUDA; ``dtype`` float64 gives an (almost) exact realisation;
``perm_seed`` permutes every conv's input channels (same sums, another rounding order).
"""
import numpy as np
import torch
import torch.nn.functional as F

def bgr_to_gray_u8(img):
    img = np.asarray(img)
    if img.ndim == 2:
        return img.astype(np.uint8)
    b, g, r = (img[..., i].astype(np.int32) for i in range(3))
    return ((b * 1868 + g * 9617 + r * 4899 + 8192) >> 14).astype(np.uint8)


def _bf16(t):
    return t.to(torch.bfloat16).to(t.dtype)


def _tf32(t):
    """Round float32 to TF32 (10 explicit mantissa bits), to nearest, ties away from zero."""
    b = t.to(torch.float32).contiguous().view(torch.int32)
    b = (b + 0x1000) & ~0x1FFF
    return b.view(torch.float32).to(t.dtype)


def simple_nms(scores, r):
    def mp(x):
        return F.max_pool2d(x, kernel_size=2 * r + 1, stride=1, padding=r)
    zeros = torch.zeros_like(scores)
    max_mask = scores == mp(scores)
    for _ in range(2):
        supp_mask = mp(max_mask.float()) > 0
        supp_scores = torch.where(supp_mask, zeros, scores)
        new_max_mask = supp_scores == mp(supp_scores)
        max_mask = max_mask | (new_max_mask & (~supp_mask))
    return torch.where(max_mask, scores, zeros)


def sample_descriptors(kp, desc, s=8):
    b, c, h, w = desc.shape
    kp = kp - s / 2 + 0.5
    kp = kp / torch.tensor([(w * s - s / 2 - 0.5), (h * s - s / 2 - 0.5)]).to(kp)[None]
    kp = kp * 2 - 1
    d = F.grid_sample(desc, kp.view(b, 1, -1, 2), mode="bilinear", align_corners=True)
    return F.normalize(d.reshape(b, c, -1), p=2, dim=1)


def dense_maps(sd, gray_f, emulate_bf16=True, sites=None, tf32=False, perm_seed=None):
    """gray_f float32 [B, 1, H, W] in [0, 1] -> (scores [B, H, W], descriptor map [B, 256, H/8, W/8]).
    Runs on gray_f's device (the CPU, or the GPU box's device when a tool uses this
    restatement as a bench-scale checker) and in gray_f's dtype."""
    sites = frozenset(("w", "act") if (sites is None and emulate_bf16) else (sites or ()))
    ident = lambda t: t  # noqa: E731
    q = _bf16 if "act" in sites else ident
    qw = _bf16 if "w" in sites else ident
    sd = {k: torch.as_tensor(np.asarray(v, np.float32)).to(gray_f.device).to(gray_f.dtype) for k, v in sd.items()}
    W = {k: (qw(v) if k.endswith("weight") and not k.startswith("conv1a") else v) for k, v in sd.items()}
    rng = None if perm_seed is None else torch.Generator().manual_seed(int(perm_seed))

    def conv(x, name, relu=True, pad=1):
        w = W[f"{name}.weight"]
        if tf32:
            x, w = _tf32(x), _tf32(w)
        if rng is not None and x.shape[1] > 1:
            p = torch.randperm(x.shape[1], generator=rng).to(x.device)
            x, w = x[:, p], w[:, p]
        y = F.conv2d(x, w, W[f"{name}.bias"], padding=pad)
        return torch.relu(y) if relu else y

    x = q(conv(gray_f, "conv1a"))
    x = q(conv(x, "conv1b"))
    x = F.max_pool2d(x, 2, 2)
    x = q(conv(x, "conv2a"))
    x = q(conv(x, "conv2b"))
    x = F.max_pool2d(x, 2, 2)
    x = q(conv(x, "conv3a"))
    x = q(conv(x, "conv3b"))
    x = F.max_pool2d(x, 2, 2)
    x = q(conv(x, "conv4a"))
    x = q(conv(x, "conv4b"))
    cPa = q(conv(x, "convPa"))
    sc = conv(cPa, "convPb", relu=False, pad=0)
    sc = F.softmax(sc, 1)[:, :-1]
    b, _, h, w = sc.shape
    sc = sc.permute(0, 2, 3, 1).reshape(b, h, w, 8, 8).permute(0, 1, 3, 2, 4).reshape(b, h * 8, w * 8)
    cDa = q(conv(x, "convDa"))
    desc = conv(cDa, "convDb", relu=False, pad=0)
    desc = F.normalize(desc, p=2, dim=1)
    return sc, desc


def detect(scores, desc, max_kp=2048, det_thr=0.001, nms_radius=4, border=4):
    """Keypoints / scores / descriptors per image from the dense maps (SuperPoint.forward tail)."""
    scores = simple_nms(scores, nms_radius)
    if border:
        scores[:, :border] = -1
        scores[:, :, :border] = -1
        scores[:, -border:] = -1
        scores[:, :, -border:] = -1
    out = []
    for i in range(scores.shape[0]):
        best = torch.where(scores[i] > det_thr)
        s = scores[i][best]
        k = torch.stack(best, -1)
        if max_kp is not None and max_kp < len(k):
            s, idx = torch.topk(s, max_kp, dim=0, sorted=True)
            k = k[idx]
        k = torch.flip(k, [1]).to(desc.dtype)
        d = sample_descriptors(k[None], desc[i:i + 1], 8)[0].T
        out.append({"keypoints": k, "keypoint_scores": s, "descriptors": d})
    return out


def superpoint(sd, images_bgr, max_kp=2048, det_thr=0.001, emulate_bf16=True, nms_radius=4, device=None, sites=None,
               tf32=False, dtype=torch.float32, perm_seed=None):
    gray = np.stack([bgr_to_gray_u8(im) for im in images_bgr]).astype(np.float32) / 255.0
    sc, desc = dense_maps(sd, torch.from_numpy(gray)[:, None].to(device or "cpu").to(dtype), emulate_bf16, sites, tf32,
                          perm_seed)
    return detect(sc, desc, max_kp, det_thr, nms_radius)
