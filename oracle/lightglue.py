"""Oracle for the LightGlue matcher (test infrastructure only).

The reference calls ``LightGlue(features='superpoint')`` (geometric_verification.py:
224-233, 285-305) from the unpinned github cvg/LightGlue HEAD, absent here with its
weights.  This is a torch-fp32 CPU restatement of its published forward pass for one
pair (batch 1, no masks), with the defaults: descriptor_dim 256, 9 layers, 4 heads,
depth_confidence 0.95, width_confidence 0.99, filter_threshold 0.1, flash attention
on CUDA (scaled_dot_product_attention), point pruning while a side has more than
1536 tokens (the CUDA + flash threshold).  Restated pieces:
  * normalize_keypoints without image_size (the reference passes bare SuperPoint
    outputs): size = 1 + max - min per image, (kpts - size/2) / (max(size)/2);
  * LearnableFourierPositionalEncoding(2, 64, 64): Wr [32, 2], cos/sin, repeated 2x
    interleaved; rotary q, k in self-attention (rotate_half on adjacent pairs);
  * SelfBlock: Wqkv unflattened as (heads, 64, 3); CrossBlock: shared to_qk, both
    directions; FFN = Linear(512,512) -> LayerNorm(512) -> GELU -> Linear(512,256),
    residual on cat([x, message]);
  * TokenConfidence sigmoid(Linear(256,1)); early stop when the confident ratio
    (pruned points count as confident) exceeds 0.95, thresholds
    clip(0.8 + 0.1 exp(-4 i / 9), 0, 1); pruning keeps matchability > 0.01 or
    confidence <= threshold;
  * MatchAssignment (final_proj / d^0.25, sigmoid_log_double_softmax) of the layer
    reached, filter_matches (mutual nearest, exp(score) > 0.1).
``emulate_bf16`` rounds every GEMM input (weights and activations) and the attention
operands to bfloat16 as the GPU kernels consume them, so GPU-vs-oracle differences
reduce to summation order.

Precision probes (tools/lg_precision_probe.py) take finer switches:
  * ``sites``: the subset of SITES whose operands are bf16-rounded (emulate_bf16 = all):
    'proj' (Wqkv / to_qk / to_v inputs + weights), 'attn' (q, k, v and P), 'out'
    (out_proj / to_out), 'ffn1' (ffn.0), 'ffn2' (ffn.3), 'asg' (final_proj);
  * ``attn_fp16``: the reference's own CUDA attention -- cvg/LightGlue's Attention.forward
    with flash enabled runs ``F.scaled_dot_product_attention`` on ``x.half()`` q, k, v and
    casts the fp16 output back (the FlashAttention kernel: fp32 scores and softmax, P
    rounded to fp16 for P.V, fp16 output);
  * ``dtype``: torch.float64 for an (almost) exact realisation;
  * ``perm_seed``: every GEMM / attention reduction taken in a seeded permuted order -- a
    second fp32 realisation with the same operands and different rounding sequence.
"""
import numpy as np
import torch
import torch.nn.functional as F

D, H, L = 256, 4, 9
HD = D // H
SITES = ("proj", "attn", "out", "ffn1", "ffn2", "asg")
_SITE_OF = {"Wqkv": "proj", "to_qk": "proj", "to_v": "proj", "out_proj": "out", "to_out": "out", "ffn.0": "ffn1",
            "ffn.3": "ffn2", "final_proj": "asg"}


def _site(name):
    for key, site in _SITE_OF.items():
        if name.endswith(key):
            return site
    raise KeyError(name)


def conf_threshold(i, n_layers=L):
    return float(np.clip(0.8 + 0.1 * np.exp(-4.0 * i / n_layers), 0, 1))


def _q(t, on):
    return t.to(torch.bfloat16).to(torch.float32) if on else t


def normalize_keypoints(k):
    size = 1 + k.max(-2).values - k.min(-2).values
    shift = size / 2
    scale = size.max(-1).values / 2
    return (k - shift[..., None, :]) / scale[..., None, None]


def rotate_half(x):
    x = x.unflatten(-1, (-1, 2))
    x1, x2 = x.unbind(dim=-1)
    return torch.stack((-x2, x1), dim=-1).flatten(start_dim=-2)


def _h(t):
    return t.to(torch.float16).to(t.dtype)


class Oracle:
    def __init__(self, sd, emulate_bf16=True, device=None, sites=None, attn_fp16=False, dtype=torch.float32,
                 perm_seed=None):
        # device: the CPU by default; a bench-scale checker tool may place the fp32
        # restatement on the GPU box's device (same ops, fp32 throughout)
        self.dev = torch.device(device or "cpu")
        self.dt = dtype
        self.sd = {k: torch.as_tensor(np.asarray(v, np.float32)).to(self.dev).to(dtype) for k, v in sd.items()}
        self.sites = frozenset(SITES if (sites is None and emulate_bf16) else (sites or ()))
        self.bf = bool(self.sites)
        self.fp16 = bool(attn_fp16)
        self.rng = None if perm_seed is None else torch.Generator().manual_seed(int(perm_seed))

    def _perm(self, n):
        return None if self.rng is None else torch.randperm(n, generator=self.rng).to(self.dev)

    def _mm(self, a, b):
        """a @ b, the reduction in a permuted order when perm_seed is set."""
        p = self._perm(a.shape[-1])
        return a @ b if p is None else a[..., p] @ b[..., p, :]

    def lin(self, x, name):
        w, b = self.sd[name + ".weight"], self.sd[name + ".bias"]
        on = _site(name) in self.sites
        return self._mm(_q(x, on), _q(w, on).T) + b

    def ffn(self, x, msg, p):
        h = self.lin(torch.cat([x, msg], -1), p + ".ffn.0")
        h = F.layer_norm(h, (2 * D,), self.sd[p + ".ffn.1.weight"], self.sd[p + ".ffn.1.bias"])
        h = F.gelu(h)
        return x + self.lin(h, p + ".ffn.3")

    def attn(self, q, k, v):
        on = "attn" in self.sites
        if self.fp16:  # FlashAttention on x.half(): fp32 scores / softmax, fp16 P and output
            q, k, v = (_h(t) for t in (q, k, v))
            s = self._mm(q, k.transpose(-1, -2)) / HD ** 0.5
            return _h(self._mm(_h(torch.softmax(s, -1)), v))
        q, k, v = (_q(t, on) for t in (q, k, v))
        s = self._mm(q, k.transpose(-1, -2)) / HD ** 0.5
        p = torch.softmax(s, -1)
        return self._mm(_q(p, on), v)

    def self_block(self, x, enc, i):
        p = f"transformers.{i}.self_attn"
        qkv = self.lin(x, p + ".Wqkv").unflatten(-1, (H, -1, 3)).transpose(0, 1)  # [H, N, 64, 3]
        q, k, v = qkv[..., 0], qkv[..., 1], qkv[..., 2]
        q = q * enc[0] + rotate_half(q) * enc[1]
        k = k * enc[0] + rotate_half(k) * enc[1]
        ctx = self.attn(q, k, v).transpose(0, 1).flatten(-2)
        return self.ffn(x, self.lin(ctx, p + ".out_proj"), p)

    def cross_block(self, x0, x1, i):
        p = f"transformers.{i}.cross_attn"
        qk0, qk1 = self.lin(x0, p + ".to_qk"), self.lin(x1, p + ".to_qk")
        v0, v1 = self.lin(x0, p + ".to_v"), self.lin(x1, p + ".to_v")
        sp = lambda t: t.unflatten(-1, (H, -1)).transpose(0, 1)  # noqa: E731
        m0 = self.attn(sp(qk0), sp(qk1), sp(v1)).transpose(0, 1).flatten(-2)
        m1 = self.attn(sp(qk1), sp(qk0), sp(v0)).transpose(0, 1).flatten(-2)
        m0, m1 = self.lin(m0, p + ".to_out"), self.lin(m1, p + ".to_out")
        return self.ffn(x0, m0, p), self.ffn(x1, m1, p)

    def posenc(self, k):
        proj = k @ self.sd["posenc.Wr.weight"].T
        c, s = torch.cos(proj), torch.sin(proj)
        return torch.stack([c, s], 0).repeat_interleave(2, dim=-1)  # [2, N, 64]

    def confidence(self, x, i):
        w, b = self.sd[f"token_confidence.{i}.token.0.weight"], self.sd[f"token_confidence.{i}.token.0.bias"]
        return torch.sigmoid(x @ w.T + b).squeeze(-1)

    def matchability(self, x, i):
        w, b = self.sd[f"log_assignment.{i}.matchability.weight"], self.sd[f"log_assignment.{i}.matchability.bias"]
        return x @ w.T + b

    def assignment(self, x0, x1, i):
        p = f"log_assignment.{i}"
        m0, m1 = self.lin(x0, p + ".final_proj"), self.lin(x1, p + ".final_proj")
        m0, m1 = m0 / D ** 0.25, m1 / D ** 0.25
        sim = self._mm(m0, m1.T)
        z0, z1 = self.matchability(x0, i), self.matchability(x1, i)
        cert = F.logsigmoid(z0) + F.logsigmoid(z1).T
        s0 = F.log_softmax(sim, 1)
        s1 = F.log_softmax(sim.T.contiguous(), 1).T
        m, n = sim.shape
        scores = sim.new_full((m + 1, n + 1), 0)
        scores[:m, :n] = s0 + s1 + cert
        scores[:-1, -1] = F.logsigmoid(-z0.squeeze(-1))
        scores[-1, :-1] = F.logsigmoid(-z1.squeeze(-1))
        return scores

    @staticmethod
    def filter_matches(scores, th):
        s = scores[:-1, :-1]
        max0, max1 = s.max(1), s.max(0)
        m0, m1 = max0.indices, max1.indices
        dev = s.device
        mutual0 = torch.arange(len(m0), device=dev) == m1[m0]
        mutual1 = torch.arange(len(m1), device=dev) == m0[m1]
        max0_exp = max0.values.exp()
        ms0 = torch.where(mutual0, max0_exp, torch.zeros((), device=dev))
        ms1 = torch.where(mutual1, ms0[m1], torch.zeros((), device=dev))
        valid0 = mutual0 & (ms0 > th)
        valid1 = mutual1 & valid0[m1]
        return torch.where(valid0, m0, -1), torch.where(valid1, m1, -1), ms0, ms1

    def match(self, kpts0, desc0, kpts1, desc1, depth_confidence=0.95, width_confidence=0.99,
              filter_threshold=0.1, pruning_min_kpts=1536, force_stop=None, band=5e-3):
        """One pair -> dict(matches [S, 2] (indices into the inputs), scores [S], stop, prune0, prune1,
        depth_band).  depth_band[i] = (lo, hi): the early-stop ratio of layer i if every token
        confidence within `band` of the threshold fell on the low / the high side -- the
        decision is numerically ambiguous when lo <= depth_confidence < hi.  force_stop = s
        replaces the early-stop test by "stop after layer s" (to compare matches when a
        bf16 kernel took the other side of an ambiguous decision)."""
        dev = self.dev
        k0 = normalize_keypoints(torch.as_tensor(kpts0, device=dev).to(self.dt))
        k1 = normalize_keypoints(torch.as_tensor(kpts1, device=dev).to(self.dt))
        x0 = torch.as_tensor(desc0, device=dev).to(self.dt).clone()
        x1 = torch.as_tensor(desc1, device=dev).to(self.dt).clone()
        m, n = len(x0), len(x1)
        e0, e1 = self.posenc(k0), self.posenc(k1)
        ind0, ind1 = torch.arange(m, device=dev), torch.arange(n, device=dev)
        prune0, prune1 = torch.ones(m, dtype=torch.long, device=dev), torch.ones(n, dtype=torch.long, device=dev)
        i = 0
        depth_band = []
        for i in range(L):
            if len(x0) == 0 or len(x1) == 0:
                break
            x0 = self.self_block(x0, e0, i)
            x1 = self.self_block(x1, e1, i)
            x0, x1 = self.cross_block(x0, x1, i)
            if i == L - 1:
                continue
            t0, t1 = self.confidence(x0, i), self.confidence(x1, i)
            if depth_confidence > 0:
                c = torch.cat([t0, t1])
                thr = conf_threshold(i)
                ratio = 1.0 - (c < thr).float().sum() / (m + n)
                depth_band.append((float(1.0 - (c < thr + band).float().sum() / (m + n)),
                                   float(1.0 - (c < thr - band).float().sum() / (m + n))))
                if (ratio > depth_confidence) if force_stop is None else (i + 1 == force_stop):
                    break
            if width_confidence > 0 and len(x0) > pruning_min_kpts:
                keep = torch.sigmoid(self.matchability(x0, i)).squeeze(-1) > 1 - width_confidence
                if depth_confidence > 0:  # upstream: no token confidences without early stopping
                    keep |= t0 <= conf_threshold(i)
                keep = torch.where(keep)[0]
                ind0, x0, e0 = ind0[keep], x0[keep], e0[:, keep]
                prune0[ind0] += 1
            if width_confidence > 0 and len(x1) > pruning_min_kpts:
                keep = torch.sigmoid(self.matchability(x1, i)).squeeze(-1) > 1 - width_confidence
                if depth_confidence > 0:  # upstream: no token confidences without early stopping
                    keep |= t1 <= conf_threshold(i)
                keep = torch.where(keep)[0]
                ind1, x1, e1 = ind1[keep], x1[keep], e1[:, keep]
                prune1[ind1] += 1
        if len(x0) == 0 or len(x1) == 0:
            return {"matches": torch.zeros(0, 2, dtype=torch.long, device=dev), "scores": torch.zeros(0, device=dev),
                    "stop": i + 1,
                    "prune0": prune0, "prune1": prune1, "depth_band": depth_band}
        scores = self.assignment(x0, x1, i)
        mm0, mm1, ms0, ms1 = self.filter_matches(scores, filter_threshold)
        valid = mm0 > -1
        a = torch.where(valid)[0]
        b = mm0[valid]
        return {"matches": torch.stack([ind0[a], ind1[b]], -1), "scores": ms0[valid], "stop": i + 1,
                "prune0": prune0, "prune1": prune1, "depth_band": depth_band}
