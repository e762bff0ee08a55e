"""Where does the bf16 ViT's descriptor error come from?  (GPU box tool)

Runs oracle.vit's fp32 forward (hub DINOv2-B/14 + GeM) on a sample of bench keyframes,
once in plain fp32 and once per configuration with bfloat16 rounding at selected sites
of the forward (the sites where the HIP kernels store bf16 operands): patch-embed input,
LN1 output (qkv GEMM input), q / k, softmax P and v, attention output (proj input), LN2
output (fc1 input), GELU output (fc2 input), and the GEMM weights.  For each, prints the
error of the pairwise cosine similarities against fp32 -- the quantity kNN ranking
flips on -- so the precision budget can be spent where it matters.

    python tools/vit_precision_probe.py [--frames 512]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-level-indoor-slam_amd")]

import bench  # noqa: E402
from mlgate import synthetic  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402
from oracle import vit as ovit  # noqa: E402

SITES = ("patch", "w", "ln1", "qk", "pv", "proj_in", "ln2", "fc2_in")


def bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


@torch.no_grad()
def forward(x, sd, sites, split=()):
    """oracle.vit.forward_tokens with bf16 rounding at `sites`; a site in `split` is
    rounded to hi + lo bf16 pairs instead (split-bf16, ~16 mantissa bits)."""
    def r(t, name):
        if name in split:
            hi = bf(t)
            return hi + bf(t - hi)
        return bf(t) if name in sites else t
    E, Hh = ovit.EMBED, ovit.HEADS
    B, _, S, _ = x.shape
    grid = S // ovit.PATCH
    w = lambda k: r(sd[k], "w") if k.endswith("weight") and ("qkv" in k or "proj.w" in k or "fc" in k) else sd[k]  # noqa
    t = F.conv2d(r(x, "patch"), r(sd["patch_embed.proj.weight"], "w"), sd["patch_embed.proj.bias"], stride=14)
    t = t.flatten(2).transpose(1, 2)
    t = torch.cat((sd["cls_token"].expand(B, -1, -1), t), 1) + ovit.interpolate_pos_embed(sd["pos_embed"], grid)
    T, hd = t.shape[1], E // Hh
    for i in range(ovit.DEPTH):
        p = f"blocks.{i}."
        h = r(F.layer_norm(t, (E,), sd[p + "norm1.weight"], sd[p + "norm1.bias"], eps=1e-6), "ln1")
        qkv = F.linear(h, w(p + "attn.qkv.weight"), sd[p + "attn.qkv.bias"])
        qkv = qkv.reshape(B, T, 3, Hh, hd).permute(2, 0, 3, 1, 4)
        q, k, v = r(qkv[0], "qk"), r(qkv[1], "qk"), r(qkv[2], "pv")
        a = ((q @ k.transpose(-2, -1)) * hd ** -0.5).softmax(-1)
        o = (r(a, "pv") @ v).transpose(1, 2).reshape(B, T, E)
        o = F.linear(r(o, "proj_in"), w(p + "attn.proj.weight"), sd[p + "attn.proj.bias"])
        t = t + o * sd[p + "ls1.gamma"]
        h = r(F.layer_norm(t, (E,), sd[p + "norm2.weight"], sd[p + "norm2.bias"], eps=1e-6), "ln2")
        h = r(F.gelu(F.linear(h, w(p + "mlp.fc1.weight"), sd[p + "mlp.fc1.bias"])), "fc2_in")
        t = t + F.linear(h, w(p + "mlp.fc2.weight"), sd[p + "mlp.fc2.bias"]) * sd[p + "ls2.gamma"]
    return ovit.gem(F.layer_norm(t, (E,), sd["norm.weight"], sd["norm.bias"], eps=1e-6)[:, 1:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    a = ap.parse_args()
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    dev = torch.device("cuda:0")
    seq, _ = bench.sequence(5000, 600)
    frames = synthetic.frames_device(seq, np.arange(a.frames), dev).cpu().numpy()
    x = torch.cat([ovit.preprocess(f) for f in frames]).to(dev)
    sd = {k: torch.from_numpy(np.asarray(v)).to(dev).float() for k, v in synthetic_state_dict(0).items()}

    def run(sites, split=()):
        return torch.cat([forward(x[b:b + 32], sd, sites, split) for b in range(0, len(x), 32)]).double()

    def sims(X):
        X = X / X.norm(dim=1, keepdim=True)
        return X @ X.T

    ref = run(())
    S0 = sims(ref)
    iu = torch.triu_indices(len(ref), len(ref), 1, device=dev)
    configs = [("all", SITES, ())] + [(s, (s,), ()) for s in SITES] + \
              [("all-but-" + s, tuple(x for x in SITES if x != s), ()) for s in SITES] + \
              [("split-all", SITES, SITES), ("split-w-only", SITES, ("w",)),
               ("split-act-only", SITES, tuple(s for s in SITES if s != "w"))]
    t0 = time.time()
    for name, sites, split in configs:
        X = run(sites, split)
        d = (sims(X) - S0)[iu[0], iu[1]].abs()
        cos = (X * ref).sum(1) / (X.norm(dim=1) * ref.norm(dim=1))
        print(json.dumps({"config": name, "sim_err_median": float(d.median()), "sim_err_p99": float(d.quantile(0.99)),
                          "sim_err_max": float(d.max()), "desc_1mcos_max": float((1 - cos).max()),
                          "s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
