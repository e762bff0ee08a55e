"""ViT-B/14 (CricaVPR descriptor path) microbenchmark for profiling (GPU box tool).

    python tools/vit_bench.py [--frames 246] [--batch 123] [--iters 2]

bench.py's synthetic keyframes through VitB14.forward_into (preprocess, 12 blocks of
LN / QKV GEMM / attention / proj GEMM / LN / fc1 / fc2, GeM) with the local features;
prints ms per keyframe and the HIP-event rates of the profiled ViT slots."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
sys.path.insert(0, ROOT)

from mlgate import _native, synthetic  # noqa: E402
from mlgate.vit import VitB14  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=246)
    ap.add_argument("--batch", type=int, default=123)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--vit", choices=("split", "bf16"), default="split",
                    help="split: the gate's split-bf16 forward (MLG_VIT_SPLIT, default); bf16: one bf16 pass")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    seq = synthetic.make_sequence(a.frames, max(2, a.frames // 4), 0)
    frames = synthetic.frames_device(seq, np.arange(a.frames), dev)
    eng = VitB14(synthetic_state_dict(0), device=dev, max_batch=a.batch, precise=a.vit == "split")
    desc = torch.empty(a.frames, 768, device=dev)
    local = torch.empty(a.frames, eng.n_local, 768, device=dev)
    eng.forward_into(frames, desc, local)
    torch.cuda.synchronize()
    L = _native.lib()
    L.mlg_prof_reset()
    L.mlg_prof_enable(0x1F)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        eng.forward_into(frames, desc, local)
    e1.record()
    torch.cuda.synchronize()
    L.mlg_prof_enable(0)
    import hashlib
    res = {"frames": a.frames, "batch": a.batch, "vit": a.vit,
           "desc_sha1": hashlib.sha1(desc.cpu().numpy().tobytes() + local.cpu().numpy().tobytes()).hexdigest()[:16], "ms_per_keyframe": round(e0.elapsed_time(e1) / a.iters / a.frames, 4)}
    for slot, name in ((0, "fc1"), (1, "fc2"), (2, "qkv"), (3, "proj"), (4, "attention")):
        ms, cnt, work = ctypes.c_double(), ctypes.c_long(), ctypes.c_double()
        L.mlg_prof_read(slot, ctypes.byref(ms), ctypes.byref(cnt))
        L.mlg_prof_read_work(slot, ctypes.byref(work))
        res[name] = {"ms_per_iter": round(ms.value / a.iters, 3),
                     "tflops": round(work.value / (ms.value * 1e9), 1) if ms.value else None}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
