"""Benchmark: CricaVPR (DINOv2-B/14 + GeM) descriptors + all-keyframes cosine-kNN floor
gate over a 5k-keyframe sequence (BASELINE.json configs[1]) on 1..8 MI355X.

One step = the whole sequence gated once: every keyframe (640x480x3 uint8 BGR,
resident in HBM) is preprocessed, run through ViT-B/14 (one forward yields both the
GeM descriptor and the cached local features, as CricaVPR.add_image needs), then all
keyframes are retrieved against all (top-k, time gap, threshold, floor decision).
Multi-GPU: frames are sharded across ranks (strong scaling: fixed total), descriptors
all-gathered over RCCL, each rank gates its own query rows.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
sys.path.insert(0, ROOT)

from mlgate import _native, retrieval  # noqa: E402
from mlgate import distributed as mdist  # noqa: E402
from mlgate.vit import VitB14  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md, no sparsity)
SLOTS = {0: "fc1_gemm", 1: "fc2_gemm", 2: "qkv_gemm", 3: "proj_gemm", 4: "attention"}
EMBED, MLP, T_TOK, DEPTH = 768, 3072, 530, 12


def slot_flops(slot, batch):
    """Algorithmic FLOPs of one launch of a profiled kernel for `batch` frames at 322^2."""
    m = batch * T_TOK
    return {0: 2.0 * m * EMBED * MLP, 1: 2.0 * m * MLP * EMBED, 2: 2.0 * m * EMBED * 3 * EMBED,
            3: 2.0 * m * EMBED * EMBED, 4: 4.0 * batch * 12 * T_TOK * T_TOK * 64}[slot]


def floors_for(n):
    """ISEC floor blocks 5/1/4/2 with 45.5/13.3/13.6/27.6 % of the keyframes."""
    cuts = np.round(np.cumsum([0.455, 0.133, 0.136]) * n).astype(int)
    f = np.full(n, 2, np.int64)
    f[:cuts[0]] = 5
    f[cuts[0]:cuts[1]] = 1
    f[cuts[1]:cuts[2]] = 4
    return f


def make_frames(idx, n_places, dev, seed=0):
    """Synthetic keyframes for global indices idx: a place's base scene (rectangles on
    black), shifted by up to +-5 px per visit, plus U[0, 30) noise.  Places recur on
    several floors (perceptual aliasing)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    rng = np.random.default_rng(seed)
    place_of = rng.integers(0, n_places, size=int(idx.max()) + 1)
    out = torch.empty(len(idx), 480, 640, 3, dtype=torch.uint8, device=dev)
    bases = {}
    for i, gi in enumerate(idx):
        p = int(place_of[gi])
        if p not in bases:
            r = np.random.default_rng(1000 + p)
            img = np.zeros((480, 640, 3), np.uint8)
            for _ in range(int(r.integers(20, 40))):
                x, y = int(r.integers(0, 580)), int(r.integers(0, 420))
                w, h = int(r.integers(20, 120)), int(r.integers(20, 120))
                img[y:y + h, x:x + w] = r.integers(60, 255, 3)
            bases[p] = torch.from_numpy(img).to(dev)
        sx, sy = (int(v) for v in rng.integers(-5, 6, 2))
        fr = torch.roll(bases[p], shifts=(sy, sx), dims=(0, 1)).to(torch.int16)
        fr = fr + torch.randint(0, 30, fr.shape, generator=g, device=dev, dtype=torch.int16)
        out[i] = fr.clamp_(0, 255).to(torch.uint8)
    return out


def cpu_baseline(budget_s=12.0):
    """The oracle port of the reference CPU path on this host's cores: CricaVPR.add_image
    (preprocess + TWO ViT-B/14 forwards at batch 1, place_recognition.py:759-779) on a
    bounded sample of keyframes, plus find_loop_closures over N = 5000 descriptors,
    amortised per keyframe."""
    from oracle import retrieval as oret
    from oracle import vit as ovit
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(0).items()}
    rng = np.random.default_rng(0)
    n_done, t_vit, t0 = 0, 0.0, time.perf_counter()
    while n_done < 32 and (time.perf_counter() - t0) < budget_s * 0.8:
        img = rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)
        s = time.perf_counter()
        tok = ovit.forward_tokens(ovit.preprocess(img), sd)
        ovit.gem(tok).numpy()
        ovit.forward_tokens(ovit.preprocess(img), sd)[:, 1:].numpy()
        t_vit += time.perf_counter() - s
        n_done += 1
    n = 5000
    X = rng.standard_normal((n, EMBED)).astype(np.float32)
    t = np.arange(n) * 0.765
    s = time.perf_counter()
    oret.find_loop_closures(X, t, floors_for(n), np.ones(n, np.uint8), 10.0, 0.5, 10, True)
    t_knn = time.perf_counter() - s
    per_kf = t_vit / n_done + t_knn / n
    return {"value": round(1.0 / per_kf, 3), "unit": "keyframes/s", "cores": threads, "kind": "port",
            "sample": f"{n_done} keyframes x (preprocess + 2 ViT-B/14 fp32 forwards, batch 1) = {t_vit:.1f} s; "
                      f"find_loop_closures N=5000 D=768 k=10 = {t_knn:.2f} s, amortised per keyframe"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--keyframes", type=int, default=5000)
    # 123 frames = 65,190 tokens = 255 M-tiles of 256: the 256x256 GEMM tiles of every
    # ViT layer (3 / 9 / 12 N-tiles) then fill 256 CUs in whole waves (99.6 %).
    ap.add_argument("--batch", type=int, default=123)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--places", type=int, default=600)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    N = args.keyframes
    lo, hi = mdist.shard(N, world, rank)
    n_local = hi - lo
    t_all = torch.from_numpy(np.arange(N) * 0.765).to(dev)
    f_all = torch.from_numpy(floors_for(N)).to(dev)
    hf_all = torch.ones(N, dtype=torch.uint8, device=dev)
    frames = make_frames(np.arange(lo, hi), args.places, dev)

    eng = VitB14(synthetic_state_dict(0), device=dev, max_batch=args.batch)
    gather = mdist.RowGather(N, EMBED, world, dev)
    desc_all = gather.out
    desc_loc = desc_all[lo:hi] if world == 1 else torch.empty(n_local, EMBED, device=dev)
    local_feats = torch.empty(n_local, eng.n_local, EMBED, dtype=torch.float32, device=dev)
    totals = torch.zeros(2, dtype=torch.int64, device=dev)
    L = _native.lib()

    def step():
        eng.forward_into(frames, desc_loc, local_feats)
        if world > 1:
            gather(desc_loc)  # RCCL all-gather of the descriptors over xGMI
        totals.zero_()
        return retrieval.knn_gate(desc_all, t_all, f_all, hf_all, 10.0, 0.5, args.k, True, q0=lo, Q=n_local,
                                  totals=totals)

    for i in range(args.warmup):
        if i == args.warmup - 1:
            _native.check(L.mlg_prof_enable(0x1F), "prof")
        step()
    torch.cuda.synchronize()
    import ctypes
    tot = {}
    for s in SLOTS:
        ms, cnt = ctypes.c_double(), ctypes.c_long()
        L.mlg_prof_read(s, ctypes.byref(ms), ctypes.byref(cnt))
        tot[s] = ms.value
    dom = max(tot, key=tot.get) if args.warmup > 0 else 0
    L.mlg_prof_reset()
    _native.check(L.mlg_prof_enable(1 << dom), "prof")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    L.mlg_prof_enable(0)
    ms, cnt = ctypes.c_double(), ctypes.c_long()
    L.mlg_prof_read(dom, ctypes.byref(ms), ctypes.byref(cnt))
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(totals)
    dt = dt_t.item()

    if rank == 0:
        avg_s = ms.value / 1e3 / max(cnt.value, 1)
        # algorithmic FLOPs of all timed launches (the last ViT batch of a step is ragged),
        # averaged per launch; achieved = that / the HIP-event average launch duration
        flops = slot_flops(dom, 1) * n_local * DEPTH * args.steps / max(cnt.value, 1)
        achieved = flops / avg_s / 1e12 if cnt.value else None
        valid, rejected = (int(x) for x in totals.cpu())
        line = {
            "metric": "keyframes gated/sec (CricaVPR DINOv2-B/14 descriptor + cosine-kNN floor gate)",
            "value": round(N * args.steps / dt, 2), "unit": "keyframes/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic 640x480x3 uint8 BGR keyframes (rectangle scenes, revisits, cross-floor aliasing); "
                    "seeded synthetic DINOv2-B/14 weights (no network for the hub checkpoint)",
            "config": {"workload": "configs[1]: CricaVPR (DINOv2-B/14 @322, GeM) descriptors + local features "
                                   "+ all-keyframes cosine-kNN (k=%d, gap 10 s, thr 0.5) + floor gate" % args.k,
                       "keyframes": N, "vit_batch": args.batch, "parallelism": f"frame-sharded x{world}",
                       "gate_valid": valid, "gate_rejected": rejected},
            "roofline": {"kernel": SLOTS[dom], "bound": "mfma",
                         "achieved": round(achieved, 2) if achieved else None,
                         "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4) if achieved else None,
                         "traffic": None, "avg_launch_us": round(avg_s * 1e6, 2), "launches": cnt.value,
                         "flops_per_launch": flops},
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
