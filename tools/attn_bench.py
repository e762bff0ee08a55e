"""LightGlue ragged attention microbenchmark (GPU box tool).

    python tools/attn_bench.py [--pairs 256] [--len 2048] [--iters 5]

Builds the flat token layout bench.py's LightGlue stage feeds k_attention_varlen
(pairs x 2 segments, 4 heads x 64), times the self and the cross task lists with HIP
events and prints achieved TFLOP/s (4 * heads * q * kv * 64 per task), plus the max
error of two sampled tasks against a float32 torch restatement.
"""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))

from mlgate import _native  # noqa: E402

H = 4


def tile_vt(V, Npad):
    """V f32 [H, Npad, 64] -> bf16 V^T tiled [H, Npad/64, 64 d, 64 keys]."""
    return V.view(H, Npad // 64, 64, 64).transpose(2, 3).contiguous().to(torch.bfloat16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--len", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--ragged", action="store_true")
    ap.add_argument("--clock", type=float, default=0.0,
                    help="seconds of back-to-back launches, then the in-kernel clock of a "
                         "tools/clock_probe_build.py library (mlg_probe_clock)")
    ap.add_argument("--exp2", action="store_true",
                    help="q in exp2 units (x log2(e) / 8, as lg_proj writes it for the current kernel)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    L = _native.lib()
    rng = np.random.default_rng(0)
    lens = (rng.integers(1, args.len + 1, 2 * args.pairs) if args.ragged else np.full(2 * args.pairs, args.len))
    offs = np.concatenate([[0], np.cumsum((lens + 63) // 64 * 64)])
    Npad = int(offs[-1])
    g = torch.Generator(device=dev).manual_seed(0)
    Qf = torch.randn(H, Npad, 64, device=dev, generator=g)
    Kf = torch.randn(H, Npad, 64, device=dev, generator=g)
    Vf = torch.randn(H, Npad, 64, device=dev, generator=g)
    qs = math.log2(math.e) / 8.0 if args.exp2 else 1.0
    Q, K, Vt = (Qf * qs).to(torch.bfloat16), Kf.to(torch.bfloat16), tile_vt(Vf, Npad)
    O = torch.zeros(Npad, H * 64, dtype=torch.bfloat16, device=dev)
    res = {"pairs": args.pairs, "len": args.len, "ragged": args.ragged}
    for kind in ("self", "cross"):
        tasks, outs = [], []
        for p in range(args.pairs):
            a, b = 2 * p, 2 * p + 1
            if kind == "self":
                tasks += [(offs[a], lens[a], offs[a], lens[a]), (offs[b], lens[b], offs[b], lens[b])]
            else:
                tasks += [(offs[a], lens[a], offs[b], lens[b]), (offs[b], lens[b], offs[a], lens[a])]
            outs += [offs[a], offs[b]]
        T = torch.tensor(np.array(tasks, np.int32), device=dev)
        OO = torch.tensor(np.array(outs, np.int32), device=dev)
        flops = sum(4.0 * H * 64 * t[1] * t[3] for t in tasks)
        st = _native.stream_of(dev)
        run = lambda: _native.check(L.mlg_op_attention_varlen(  # noqa: E731
            _native.ptr(Q), _native.ptr(K), _native.ptr(Vt), _native.ptr(O), H * 64, Npad, H, _native.ptr(T),
            _native.ptr(OO), len(tasks), int(lens.max()), st), "attention")
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        # numerics of two sampled tasks vs float32 softmax(q k^T / 8) v on the bf16 operands
        err = 0.0
        for ti in (0, len(tasks) - 1):
            qo, ql, ko, kl = (int(x) for x in tasks[ti])
            q = Q[:, qo:qo + ql].float()
            k = K[:, ko:ko + kl].float()
            v = Vt.float().transpose(2, 3).reshape(H, Npad, 64)[:, ko:ko + kl]
            sc = q @ k.transpose(1, 2) * (math.log(2.0) if args.exp2 else 0.125)
            ref = torch.softmax(sc, -1) @ v
            got = O[int(outs[ti]):int(outs[ti]) + ql].float().view(ql, H, 64).transpose(0, 1)
            err = max(err, float((got - ref).abs().max()))
        res[kind] = {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1), "max_abs_err": err}
        if args.clock > 0:
            import ctypes
            import time
            t_end = time.time() + args.clock
            while time.time() < t_end:
                for _ in range(10):
                    run()
                torch.cuda.synchronize()
            ghz, n = ctypes.c_double(0.0), ctypes.c_int(0)
            rc = L.mlg_probe_clock(ctypes.byref(ghz), ctypes.byref(n))
            res[kind]["clock_ghz"] = round(ghz.value, 3) if rc == 0 else None
            res[kind]["clock_wgs"] = n.value
            if rc == 0:  # TFLOP/s per GHz: the issue efficiency with the clock taken out
                res[kind]["tflops_at_2.4"] = round(flops / ms / 1e9 * 2.4 / ghz.value, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
