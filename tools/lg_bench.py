"""LightGlue stage microbenchmark (GPU box tool).

    python tools/lg_bench.py [--pairs 256] [--frames 64] [--iters 3] [--no-prune]

SuperPoint features of bench.py's synthetic keyframes, then LightGlue on `pairs`
random pairs in one call (bench.py's lg_chunk), timed with HIP events; prints the
wall time per call, the profiled slots (LightGlue attention, projections, fused FFN)
with achieved TFLOP/s (TB/s for the HBM-bound FFN), and a histogram of the layers run.
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
sys.path.insert(0, ROOT)

from mlgate import _native, synthetic  # noqa: E402
from mlgate.lightglue import LightGlueGPU  # noqa: E402
from mlgate.superpoint import SuperPointGPU  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--no-prune", action="store_true")
    ap.add_argument("--clock", type=float, default=0.0,
                    help="seconds of back-to-back calls, then the in-kernel clocks of a "
                         "tools/clock_probe_build.py library (attention, fused FFN, projections)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    seq = synthetic.make_sequence(args.frames, max(2, args.frames // 4), 0)
    frames = synthetic.frames_device(seq, np.arange(args.frames), dev)
    kp, _, ds, _, cnt = SuperPointGPU(device=dev, max_num_keypoints=2048).extract_device(frames)
    counts = cnt.cpu().numpy()
    rng = np.random.default_rng(0)
    pa = rng.integers(0, args.frames, args.pairs).astype(np.int32)
    pb = ((pa + rng.integers(1, args.frames, args.pairs)) % args.frames).astype(np.int32)
    kw = dict(depth_confidence=-1, width_confidence=-1) if args.no_prune else {}
    lg = LightGlueGPU(device=dev, **kw)
    L = _native.lib()
    m, s, n, stop = lg.match_device(kp, ds, counts, pa, pb)  # warm-up
    torch.cuda.synchronize()
    L.mlg_prof_reset()
    L.mlg_prof_enable((1 << 5) | (1 << 6) | (1 << 8))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        m, s, n, stop = lg.match_device(kp, ds, counts, pa, pb)
    e1.record()
    torch.cuda.synchronize()
    L.mlg_prof_enable(0)
    res = {"pairs": args.pairs, "mean_keypoints": float(counts.mean()), "no_prune": args.no_prune,
           "ms_per_call": round(e0.elapsed_time(e1) / args.iters, 2),
           "stop_hist": np.bincount(stop, minlength=10).tolist(), "matches_mean": float(n.float().mean()),
           # bit-identity check across builds: a digest of every pair's matches and scores
           "digest": hashlib.sha1(m.cpu().numpy().tobytes() + s.cpu().numpy().tobytes()
                                  + n.cpu().numpy().tobytes()).hexdigest()[:16]}
    for slot, name in ((5, "attention"), (6, "qkv_proj"), (8, "ffn_fused")):
        ms, cnt_, work = ctypes.c_double(), ctypes.c_long(), ctypes.c_double()
        L.mlg_prof_read(slot, ctypes.byref(ms), ctypes.byref(cnt_))
        L.mlg_prof_read_work(slot, ctypes.byref(work))
        rate = work.value / (ms.value * 1e9) if ms.value else None  # TFLOP/s (slot 8 is priced in FLOPs too)
        res[name] = {"ms_per_call": round(ms.value / args.iters, 2), "tflops": round(rate, 2) if rate else None}
    if args.clock > 0:
        import time
        t_end = time.time() + args.clock
        while time.time() < t_end:
            lg.match_device(kp, ds, counts, pa, pb)
            torch.cuda.synchronize()
        for name, fn in (("attention", "mlg_probe_clock"), ("ffn_fused", "mlg_probe_clock_ffn"),
                         ("qkv_proj", "mlg_probe_clock_proj")):
            ghz, nwg = ctypes.c_double(0.0), ctypes.c_int(0)
            rc = getattr(L, fn)(ctypes.byref(ghz), ctypes.byref(nwg))
            res[name]["clock_ghz"] = round(ghz.value, 3) if rc == 0 else None
            res[name]["clock_wgs"] = nwg.value
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
