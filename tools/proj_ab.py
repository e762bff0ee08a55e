"""LightGlue projection / FFN kernels vs the generic persistent GEMM at the same shapes
(GPU box tool): HIP-event times per launch.

    python tools/proj_ab.py [--tokens 2097152] [--iters 5]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
from mlgate import _native  # noqa: E402


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        rc = fn()
        assert rc == 0, rc
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=1 << 21)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    L = _native.lib()
    dev = torch.device("cuda:0")
    M = a.tokens
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device=dev).manual_seed(0)
    bf = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.1).to(torch.bfloat16)  # noqa: E731
    f32 = lambda *s: torch.randn(*s, device=dev, generator=g) * 0.1  # noqa: E731
    cat = bf(M, 512)
    ctx = bf(M, 256)
    X = f32(M, 256)
    Wqkv, bqkv = bf(768 * 256), f32(768)
    Wo, bo, W1, b1, W2, b2 = bf(256 * 256), f32(256), bf(512 * 512), f32(512), bf(256 * 512), f32(256)
    lng, lnb = f32(512) + 1, f32(512)
    ec, es = f32(M, 64), None  # the lg_fac4 factor block (values do not matter for timing)
    live = torch.ones(M, dtype=torch.uint8, device=dev)
    Q, K, Vt = bf(4 * M * 64), bf(4 * M * 64), bf(4 * M * 64)
    out = torch.empty(M, 768, dtype=torch.bfloat16, device=dev)
    out512 = torch.empty(M, 512, dtype=torch.bfloat16, device=dev)
    res = {"tokens": M}
    res["lg_proj_self_ms"] = timeit(lambda: L.mlg_op_lg_proj(1, p(cat), 512, p(Wqkv), p(bqkv), p(ec), None, p(live),
                                                             p(Q), p(K), p(Vt), M, st), a.iters)
    res["lg_proj_cross_ms"] = timeit(lambda: L.mlg_op_lg_proj(0, p(cat), 512, p(Wqkv), p(bqkv), None, None, p(live),
                                                              p(Q), None, p(Vt), M, st), a.iters)
    A256 = cat[:, :256].contiguous()
    res["gemm_768x256_gelu_ms"] = timeit(lambda: L.mlg_op_gemm_bias_gelu(p(A256), p(Wqkv), p(bqkv), p(out), M, 768,
                                                                         256, st), a.iters)
    res["gemm_512x512_gelu_ms"] = timeit(lambda: L.mlg_op_gemm_bias_gelu(p(cat), p(W1), p(b1), p(out512), M, 512, 512,
                                                                         st), a.iters)
    res["lg_ffn_ms"] = timeit(lambda: L.mlg_op_lg_ffn(p(ctx), p(X), p(cat), 512, M, p(Wo), p(bo), p(W1), p(b1),
                                                      p(lng), p(lnb), p(W2), p(b2), st), a.iters)
    for k in ("lg_proj_self_ms", "gemm_768x256_gelu_ms"):
        res[k.replace("_ms", "_tflops")] = round(2 * M * 768 * 256 / res[k] / 1e9, 1)
    res["lg_proj_cross_tflops"] = round(2 * M * 512 * 256 / res["lg_proj_cross_ms"] / 1e9, 1)
    res["gemm_512x512_gelu_tflops"] = round(2 * M * 512 * 512 / res["gemm_512x512_gelu_ms"] / 1e9, 1)
    res["lg_ffn_tflops"] = round(917504 * M / res["lg_ffn_ms"] / 1e9, 1)
    res["lg_ffn_tbps"] = round(3584 * M / res["lg_ffn_ms"] / 1e9, 2)
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
