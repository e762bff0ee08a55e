"""Oracle for the SALAD descriptor path (test infrastructure only).

Reference: ``SALAD`` (place_recognition.py:335-410).  Its native branch builds
``salad.SALAD(out_dim=descriptor_dim)`` (:357-368) and runs ``self.model(tensor)`` on
``_preprocess`` output (:380-391); the package is not installed anywhere this runs, so
the reference executes the MixVPR fallback (:370-378) and the native
branch is unpinned.  What that branch names is serizba/salad (``models/aggregators/
salad.py``, published with the paper "Optimal Transport Aggregation for Visual Place
Recognition"): a DINOv2 ViT-B/14 backbone whose final-LayerNorm tokens feed

  * ``token_features``   Linear(768, 512) - ReLU - Linear(512, 256) on the CLS token,
  * ``cluster_features`` Conv1x1(768, 512) - Dropout - ReLU - Conv1x1(512, 128),
  * ``score``            Conv1x1(768, 512) - Dropout - ReLU - Conv1x1(512, 64),
  * ``get_matching_probs``: the score matrix [64, n] augmented with a dustbin row of
    the learned ``dust_bin`` value, log-domain Sinkhorn (``log_otp_solver``, reg 1,
    3 iterations) between log-marginals a = -log(n + m) (dustbin row + log(n - m)) and
    b = -log(n + m), minus the normaliser, exponentiated, dustbin dropped,
  * aggregation  sum_n f[l, n] p[c, n] -> [128, 64], L2-normalised over l per cluster,
    flattened l-major (index l * 64 + c), appended to the L2-normalised token
    features, and the 8448-vector L2-normalised.

Input: the DINOv2 PatchEmbed asserts H % 14 == W % 14 == 0, so the reference's
``cv2.resize(image, (480, 640))`` (:395) cannot enter the hub backbone; this path (and
the GPU path) resizes to SALAD's published evaluation size 322 x 322 with cv2
INTER_LINEAR and otherwise keeps the reference's preprocessing: no channel swap
(only GRAY -> RGB, :396-397), float32 / 255, float64 ImageNet normalisation, float32.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import vit as _vit

NUM_CLUSTERS, CLUSTER_DIM, TOKEN_DIM = 64, 128, 256
DESC_DIM = NUM_CLUSTERS * CLUSTER_DIM + TOKEN_DIM  # 8448
IMAGE_SIZE = 322


def _t(sd, k):
    v = sd[k]
    return (v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))).float()


def backbone_state_dict(sd):
    """The hub dinov2 keys of a SALAD state dict (``backbone.model.`` prefix stripped)."""
    p = "backbone.model."
    return {k[len(p):]: v for k, v in sd.items() if k.startswith(p)}


def log_otp_solver(log_a, log_b, M, num_iters, reg=1.0):
    """serizba/salad log_otp_solver: alternating u / v log-sum-exp updates."""
    M = M / reg
    u, v = torch.zeros_like(log_a), torch.zeros_like(log_b)
    for _ in range(num_iters):
        u = log_a - torch.logsumexp(M + v.unsqueeze(1), dim=2).squeeze()
        v = log_b - torch.logsumexp(M + u.unsqueeze(2), dim=1).squeeze()
    return M + u.unsqueeze(2) + v.unsqueeze(1)


def get_matching_probs(S, dustbin_score, num_iters=3, reg=1.0):
    """serizba/salad get_matching_probs: [B, m, n] scores -> log P [B, m + 1, n]."""
    B, m, n = S.shape
    S_aug = torch.empty(B, m + 1, n, dtype=S.dtype)
    S_aug[:, :m, :n] = S
    S_aug[:, m, :] = dustbin_score
    norm = -torch.tensor(math.log(n + m))
    log_a, log_b = norm.expand(m + 1).contiguous(), norm.expand(n).contiguous()
    log_a[-1] = log_a[-1] + math.log(n - m)
    log_a, log_b = log_a.expand(B, -1), log_b.expand(B, -1)
    log_P = log_otp_solver(log_a, log_b, S_aug, num_iters=num_iters, reg=reg)
    return log_P - norm


@torch.no_grad()
def aggregate(tokens, sd):
    """SALAD.forward on final-LayerNorm tokens [B, 1 + n, 768] -> [B, 8448]."""
    a = "aggregator."
    t, x = tokens[:, 0], tokens[:, 1:]
    h = F.relu(F.linear(x, _t(sd, a + "cluster_features.0.weight").flatten(1), _t(sd, a + "cluster_features.0.bias")))
    f = F.linear(h, _t(sd, a + "cluster_features.3.weight").flatten(1), _t(sd, a + "cluster_features.3.bias"))
    h = F.relu(F.linear(x, _t(sd, a + "score.0.weight").flatten(1), _t(sd, a + "score.0.bias")))
    p = F.linear(h, _t(sd, a + "score.3.weight").flatten(1), _t(sd, a + "score.3.bias"))
    f, p = f.transpose(1, 2), p.transpose(1, 2)  # [B, 128, n], [B, 64, n] (conv output flatten(2))
    tt = F.linear(F.relu(F.linear(t, _t(sd, a + "token_features.0.weight"), _t(sd, a + "token_features.0.bias"))),
                  _t(sd, a + "token_features.2.weight"), _t(sd, a + "token_features.2.bias"))
    p = torch.exp(get_matching_probs(p, _t(sd, a + "dust_bin"), 3))[:, :-1, :]
    agg = torch.einsum("bln,bcn->blc", f, p)  # == (f.unsqueeze(2) * p.unsqueeze(1)).sum(-1)
    out = torch.cat([F.normalize(tt, p=2, dim=-1), F.normalize(agg, p=2, dim=1).flatten(1)], dim=-1)
    return F.normalize(out, p=2, dim=-1)


@torch.no_grad()
def extract_descriptor(image, sd):
    """SALAD.extract_descriptor native branch -> float32 (8448,)."""
    x = _vit.preprocess(image, IMAGE_SIZE, swap_rb=False)
    return aggregate(_vit.forward_tokens_with_cls(x, backbone_state_dict(sd)), sd).cpu().numpy().flatten()
