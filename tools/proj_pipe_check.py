"""LightGlue projections (lg_proj.hip) on seeded inputs with a ragged live mask, and the
fused block tail (lg_ffn.hip): sha1 of Q / K / V^T, of the updated residual X and its
bf16 copy, and HIP-event ms per launch, for same-box A/B of two builds through
tools/ab_run.py (GPU box tool; the arms must print the same hashes).

    python tools/proj_pipe_check.py [--tokens 2097152] [--iters 10]
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
from mlgate import _native  # noqa: E402


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=1 << 21)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    L = _native.lib()
    dev = torch.device("cuda:0")
    M = a.tokens
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device=dev).manual_seed(0)
    cat = (torch.randn(M, 512, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    W = (torch.randn(768 * 256, device=dev, generator=g) * 0.06).to(torch.bfloat16)
    b = torch.randn(768, device=dev, generator=g) * 0.1
    ang = torch.rand(M, 32, device=dev, generator=g) * 6.283
    from mlgate.lightglue import pack_rotary
    ec = pack_rotary(torch.cos(ang), torch.sin(ang))
    live = (torch.rand(M, device=dev, generator=g) < 0.85).to(torch.uint8)
    res = {"tokens": M}
    for name, sb in (("self", 1), ("cross", 0)):
        Q = torch.full((4 * M * 64,), 7, dtype=torch.int16, device=dev)
        K = torch.full_like(Q, 7)
        Vt = torch.full_like(Q, 7)
        fn = lambda: L.mlg_op_lg_proj(sb, p(cat), 512, p(W), p(b), p(ec) if sb else None,  # noqa: E731
                                      None, p(live), p(Q), p(K) if sb else None, p(Vt), M, st)
        assert fn() == 0
        torch.cuda.synchronize()
        h = hashlib.sha1()
        for t in ((Q, K, Vt) if sb else (Q, Vt)):
            h.update(t.cpu().numpy().tobytes())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        n = 768 if sb else 512
        res[name] = {"sha1": h.hexdigest()[:16], "ms": round(ms, 3), "tflops": round(2 * M * n * 256 / ms / 1e9, 1)}
    # fused block tail: x += FFN([x | out_proj(ctx)]) on the same cat / live rows
    ctx = (torch.randn(M, 256, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    X0 = torch.randn(M, 256, device=dev, generator=g)
    bf = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.05).to(torch.bfloat16)  # noqa: E731
    f32 = lambda *s: torch.randn(*s, device=dev, generator=g) * 0.1  # noqa: E731
    Wo, bo, W1, b1, W2, b2 = bf(256 * 256), f32(256), bf(512 * 512), f32(512), bf(256 * 512), f32(256)
    lng, lnb = f32(512) + 1, f32(512)
    X = X0.clone()
    cat2 = cat.clone()
    ffn = lambda: L.mlg_op_lg_ffn(p(ctx), p(X), p(cat2), 512, M, p(Wo), p(bo), p(W1), p(b1),  # noqa: E731
                                  p(lng), p(lnb), p(W2), p(b2), st)
    assert ffn() == 0
    torch.cuda.synchronize()
    h = hashlib.sha1()
    h.update(X.cpu().numpy().tobytes())
    h.update(cat2.view(torch.int16).cpu().numpy().tobytes())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        ffn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    res["ffn"] = {"sha1": h.hexdigest()[:16], "ms": round(ms, 3), "tflops": round(917504 * M / ms / 1e9, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
