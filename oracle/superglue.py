"""Oracle for the SuperGlue matcher (test infrastructure only).

The reference's ``SuperGlue`` class (scripts/semantic_gating/geometric_verification.py:
353-421) configures magicleap's SuperGluePretrainedNetwork (cloned unpinned by
docker/Dockerfile.semantic-tools:88-90, absent here with its weights) as
``SG({'weights': 'indoor', 'sinkhorn_iterations': 20, 'match_threshold': 0.2})`` and then
never calls it (its native branch returns the LightGlue fallback, :419-421).  This is a
torch-fp32 CPU restatement of that model's published forward pass for one pair, from the
raw (unfolded, channel-interleaved) state dict:
  * normalize_keypoints: (kpts - size / 2) / (0.7 max(size)), size = (W, H) of the image;
  * KeypointEncoder: MLP [3, 32, 64, 128, 256, 256] over (x, y, score), Conv1d(k=1) +
    eval BatchNorm1d + ReLU on every layer but the last; desc + kenc;
  * AttentionalGNN: 18 layers ['self', 'cross'] * 9; MultiHeadedAttention (4 heads,
    head h's dim d on channel d * 4 + h, softmax(q k^T / sqrt(64))), merge; message
    MLP [512, 512, 256] on cat([x, message]); both sides updated from the pre-layer states;
  * final_proj, scores = m0^T m1 / sqrt(256), log_optimal_transport with the learned
    bin_score (dustbin row / column / corner), 20 log-Sinkhorn iterations, Z - norm;
  * mutual nearest over the inner [m, n] block, exp(max) > match_threshold.
Parity: UNPINNED against magicleap itself (package and weights absent, no golden
vectors in the reference); pinned by the Sinkhorn marginal identities and the tests in
tests/test_oracle_superglue.py.  ``emulate_bf16`` rounds the activations entering every
GEMM / attention product to bfloat16 as the GPU kernels consume them.
"""
import numpy as np
import torch

D, HEADS, LAYERS = 256, 4, 18


def _t(a):
    return torch.as_tensor(np.asarray(a, np.float32))


def _q(t, on):
    return t.to(torch.bfloat16).to(torch.float32) if on else t


def normalize_keypoints(kpts, width, height):
    size = torch.tensor([float(width), float(height)])
    return (kpts - size / 2) / (size.max() * 0.7)


def _conv(sd, name, x, bf=False):
    """Conv1d(k=1) on channel-last rows x [n, cin] -> [n, cout]."""
    return _q(x, bf) @ _t(sd[name + ".weight"])[:, :, 0].T + _t(sd[name + ".bias"])


def _bn(sd, name, x, eps=1e-5):
    return (x - _t(sd[name + ".running_mean"])) / torch.sqrt(_t(sd[name + ".running_var"]) + eps) * _t(
        sd[name + ".weight"]) + _t(sd[name + ".bias"])


def keypoint_encoder(sd, kpts, scores, width, height, emulate_bf16=False):
    x = torch.cat([normalize_keypoints(kpts, width, height), scores[:, None]], 1)
    for i in range(5):
        x = _conv(sd, f"kenc.encoder.{3 * i}", x, emulate_bf16 and i >= 3)
        if i < 4:
            x = torch.relu(_bn(sd, f"kenc.encoder.{3 * i + 1}", x))
    return x


def attention(q, k, v, emulate_bf16=False):
    """Rows [n, 256] with channel d * 4 + h -> message rows [n, 256] (same interleave)."""
    n, m = q.shape[0], k.shape[0]
    qh, kh, vh = (t.reshape(t.shape[0], 64, HEADS).permute(2, 0, 1) for t in (q, k, v))  # [h, n, 64]
    s = torch.einsum("hnd,hmd->hnm", _q(qh, emulate_bf16), _q(kh, emulate_bf16)) / 64 ** 0.5
    p = torch.softmax(s, -1)
    o = torch.einsum("hnm,hmd->hnd", _q(p, emulate_bf16), _q(vh, emulate_bf16))  # [h, n, 64]
    return o.permute(1, 2, 0).reshape(n, D)


def propagate(sd, p, x, src, emulate_bf16=False):
    """AttentionalPropagation: delta = mlp(cat([x, attn(x, src, src)]))."""
    q = _conv(sd, p + "attn.proj.0", x, emulate_bf16)
    k = _conv(sd, p + "attn.proj.1", src, emulate_bf16)
    v = _conv(sd, p + "attn.proj.2", src, emulate_bf16)
    msg = _conv(sd, p + "attn.merge", attention(q, k, v, emulate_bf16), emulate_bf16)
    h = torch.relu(_bn(sd, p + "mlp.1", _conv(sd, p + "mlp.0", torch.cat([x, msg], 1), emulate_bf16)))
    return _conv(sd, p + "mlp.3", h, emulate_bf16)


def gnn(sd, d0, d1, emulate_bf16=False):
    for i in range(LAYERS):
        p = f"gnn.layers.{i}."
        s0, s1 = (d1, d0) if i % 2 else (d0, d1)
        e0, e1 = propagate(sd, p, d0, s0, emulate_bf16), propagate(sd, p, d1, s1, emulate_bf16)
        d0, d1 = d0 + e0, d1 + e1
    return d0, d1


def log_optimal_transport(scores, alpha, iters):
    """scores [m, n] -> log assignment [m + 1, n + 1] (dustbins last), times (m + n)."""
    m, n = scores.shape
    alpha = torch.as_tensor(alpha, dtype=scores.dtype)
    Z = torch.cat([torch.cat([scores, alpha.expand(m, 1)], 1), alpha.expand(1, n + 1)], 0)
    norm = -torch.log(torch.tensor(float(m + n)))
    log_mu = torch.cat([norm.expand(m), (torch.log(torch.tensor(float(n))) + norm)[None]])
    log_nu = torch.cat([norm.expand(n), (torch.log(torch.tensor(float(m))) + norm)[None]])
    u, v = torch.zeros_like(log_mu), torch.zeros_like(log_nu)
    for _ in range(iters):
        u = log_mu - torch.logsumexp(Z + v[None, :], 1)
        v = log_nu - torch.logsumexp(Z + u[:, None], 0)
    return Z + u[:, None] + v[None, :] - norm


def mutual_matches(P, threshold):
    """Inner block of the log assignment -> (matches0 [m] or -1, mscores0 [m])."""
    inner = P[:-1, :-1]
    max0, idx0 = inner.max(1)
    _, idx1 = inner.max(0)
    mutual0 = torch.arange(inner.shape[0]) == idx1[idx0]
    ms0 = torch.where(mutual0, max0.exp(), torch.zeros(()))
    valid0 = mutual0 & (ms0 > threshold)
    return torch.where(valid0, idx0, torch.full_like(idx0, -1)), ms0


class Oracle:
    """SuperGlue for one pair from a magicleap-style state dict (numpy values)."""

    def __init__(self, sd, sinkhorn_iterations=20, match_threshold=0.2, emulate_bf16=False):
        self.sd = sd
        self.iters = sinkhorn_iterations
        self.thr = match_threshold
        self.bf = emulate_bf16

    def descriptors(self, kpts0, scores0, desc0, kpts1, scores1, desc1, width, height):
        """Matching descriptors (final_proj output) [m, 256], [n, 256]."""
        sd, bf = self.sd, self.bf
        d0 = _t(desc0) + keypoint_encoder(sd, _t(kpts0), _t(scores0), width, height, bf)
        d1 = _t(desc1) + keypoint_encoder(sd, _t(kpts1), _t(scores1), width, height, bf)
        d0, d1 = gnn(sd, d0, d1, bf)
        return _conv(sd, "final_proj", d0, bf), _conv(sd, "final_proj", d1, bf)

    def log_assignment(self, m0, m1):
        scores = (m0 @ m1.T) / D ** 0.5
        return log_optimal_transport(scores, float(np.asarray(self.sd["bin_score"])), self.iters)

    def match(self, kpts0, scores0, desc0, kpts1, scores1, desc1, width, height):
        """-> (matches [S, 2] int (i, j) in row order, scores [S] float32)."""
        if len(kpts0) == 0 or len(kpts1) == 0:
            return np.zeros((0, 2), np.int64), np.zeros(0, np.float32)
        with torch.no_grad():
            m0, m1 = self.descriptors(kpts0, scores0, desc0, kpts1, scores1, desc1, width, height)
            idx0, ms0 = mutual_matches(self.log_assignment(m0, m1), self.thr)
        i = torch.nonzero(idx0 >= 0)[:, 0]
        return torch.stack([i, idx0[i]], 1).numpy(), ms0[i].numpy().astype(np.float32)
