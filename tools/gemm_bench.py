"""Per-kernel timing of the ViT-B/14 forward for each GEMM generation (GPU box tool).

    python tools/gemm_bench.py [--batch 64] [--iters 5]

Prints one JSON line per variant with the average HIP-event duration and achieved
TFLOP/s of every profiled kernel slot, plus a bit-exactness check of the variants.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))

from mlgate import _native  # noqa: E402
from mlgate.vit import VitB14  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402

SLOTS = {0: "fc1", 1: "fc2", 2: "qkv", 3: "proj", 4: "attention"}


def flops(slot, b):
    m = b * 530
    return {0: 2 * m * 768 * 3072, 1: 2 * m * 3072 * 768, 2: 2 * m * 768 * 2304, 3: 2 * m * 768 * 768,
            4: 4 * b * 12 * 530 * 530 * 64}[slot]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--variants", default="2,3,4")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    L = _native.lib()
    # bit-exactness of the GEMM generations on a ragged shape
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.randn(33920 - 17, 768, device=dev, generator=g).to(torch.bfloat16)
    W = torch.randn(3072, 768, device=dev, generator=g).to(torch.bfloat16)
    outs = {}
    for v in (1, 2, 3, 4, 5):
        C = torch.empty(A.shape[0], 3072, device=dev)
        _native.check(L.mlg_op_gemm_f32out_variant(v, _native.ptr(A), _native.ptr(W), _native.ptr(C), A.shape[0],
                                                   3072, 768, _native.stream_of(dev)), "gemm")
        outs[v] = C
    torch.cuda.synchronize()
    print(json.dumps({"variants_bit_identical": all(bool(torch.equal(outs[1], outs[v])) for v in (2, 3, 4, 5))}),
          flush=True)

    # loop throughput vs fixed per-tile cost: time C = A W^T (f32 out) at K = 768 .. 6144
    for v in (4, 5):
        row = {"variant": v, "M": 33920, "N": 3072}
        for K in (768, 1536, 3072, 6144):
            A = torch.randn(33920, K, device=dev, generator=g).to(torch.bfloat16)
            W = torch.randn(3072, K, device=dev, generator=g).to(torch.bfloat16)
            C = torch.empty(33920, 3072, device=dev)
            args_ = (v, _native.ptr(A), _native.ptr(W), _native.ptr(C), 33920, 3072, K, _native.stream_of(dev))
            L.mlg_op_gemm_f32out_variant(*args_)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                L.mlg_op_gemm_f32out_variant(*args_)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 100.0
            row[f"K{K}_us"] = round(us, 1)
            row[f"K{K}_tflops"] = round(2 * 33920 * 3072 * K / us / 1e6, 1)
        print(json.dumps(row), flush=True)

    # LightGlue shapes: ~1M token rows, K = 256 / 512 (per-variant f32-out timing)
    for (N, K) in ((768, 256), (512, 512), (256, 512), (256, 256)):
        M = 1 << 20
        A = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        W = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev)
        row = {"lightglue_shape": [M, N, K]}
        for v in (1, 2, 4):
            args_ = (v, _native.ptr(A), _native.ptr(W), _native.ptr(C), M, N, K, _native.stream_of(dev))
            L.mlg_op_gemm_f32out_variant(*args_)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                L.mlg_op_gemm_f32out_variant(*args_)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 200.0
            row[f"v{v}_us"] = round(us, 1)
            row[f"v{v}_tflops"] = round(2.0 * M * N * K / us / 1e6, 1)
        print(json.dumps(row), flush=True)
        del A, W, C

    eng = VitB14(synthetic_state_dict(0), device=dev, max_batch=args.batch, precise=False)
    frames = torch.randint(0, 256, (args.batch, 480, 640, 3), dtype=torch.uint8, device=dev)
    desc = {}
    for v in (int(x) for x in args.variants.split(",")):
        _native.check(L.mlg_set_gemm_variant(v), "variant")
        eng.forward(frames)
        torch.cuda.synchronize()
        L.mlg_prof_reset()
        _native.check(L.mlg_prof_enable(0x1F), "prof")
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(args.iters):
            d = eng.forward(frames)
        t1.record()
        torch.cuda.synchronize()
        L.mlg_prof_enable(0)
        res = {"variant": v, "forward_ms": t0.elapsed_time(t1) / args.iters,
               "keyframes_per_s": args.batch * args.iters / (t0.elapsed_time(t1) / 1e3)}
        for s, name in SLOTS.items():
            ms, cnt = ctypes.c_double(), ctypes.c_long()
            L.mlg_prof_read(s, ctypes.byref(ms), ctypes.byref(cnt))
            avg = ms.value / max(cnt.value, 1)
            res[name] = {"avg_us": round(avg * 1e3, 2), "tflops": round(flops(s, args.batch) / (avg / 1e3) / 1e12, 1)}
        desc[v] = d.clone()
        print(json.dumps(res), flush=True)
    if len(desc) > 1:
        vs = list(desc)
        print(json.dumps({"descriptors_equal": bool(torch.equal(desc[vs[0]], desc[vs[1]]))}))


if __name__ == "__main__":
    main()
