"""Benchmark: the semantic loop-closure gate -- CricaVPR (DINOv2-B/14 + GeM) descriptors,
all-keyframes cosine-kNN floor gate, and SuperPoint + LightGlue + RANSAC verification of
the gate-accepted candidates -- over a 5k-keyframe sequence on 1..8 MI355X
(BASELINE.json metric "keyframes gated/sec (VPR+kNN+LightGlue verify)"; workload
configs[1] descriptors + kNN, verified as in configs[2]).

One step = the whole sequence gated once: every keyframe (640x480x3 uint8 BGR,
resident in HBM) is preprocessed and run through ViT-B/14 (one forward yields the GeM
descriptor and the cached local features, as CricaVPR.add_image needs); all keyframes
are retrieved against all (top-k, time gap, threshold, floor decision); every
candidate the floor gate accepts is verified: SuperPoint keypoints / descriptors per
keyframe (computed once, cached), LightGlue on the pair, essential-matrix RANSAC +
recoverPose, and the verifier's decision rule (>= 20 inliers, ratio >= 0.25).
Multi-GPU: frames are sharded across ranks (strong scaling: fixed total); descriptors
and SuperPoint features are all-gathered over RCCL; each rank gates its own query rows,
then the gate-accepted pairs are all-gathered and re-split evenly for verification.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--verify all|none]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import ctypes
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

from mlgate import _native, geometry, retrieval  # noqa: E402
from mlgate import distributed as mdist  # noqa: E402
from mlgate.lightglue import LightGlueGPU  # noqa: E402
from mlgate.superpoint import SuperPointGPU  # noqa: E402
from mlgate.vit import VitB14  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md, no sparsity)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
SLOTS = {0: "vit_fc1_gemm", 1: "vit_fc2_gemm", 2: "vit_qkv_gemm", 3: "vit_proj_gemm", 4: "vit_attention",
         5: "lightglue_attention", 6: "lightglue_qkv_gemms", 7: "superpoint_conv3x3", 8: "lightglue_ffn_fused"}
HBM_SLOTS = {8}  # slots whose recorded work is algorithmic HBM bytes (bound "hbm"), not FLOPs
EMBED, KP = 768, 2048
ISEC_K = np.array([[893.63, 0.0, 376.95], [0.0, 893.97, 266.57], [0.0, 0.0, 1.0]])  # cam1, SURVEY §8


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


def pmc_traffic(slot_name):
    """HBM bytes per launch of the dominant kernel from the committed PMC pass
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from separate
    `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` runs of this bench, with the
    gfx950 FETCH_SIZE x2 correction of MI355X_MICROARCH.md), or None if absent."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        entry = json.load(f).get(slot_name)
    return entry.get("bytes_per_launch") if entry else None


def cpu_baseline(budget_s=12.0, pairs_per_kf=0.0):
    """The oracle port of the reference CPU path on this host's cores, per keyframe:
    CricaVPR.add_image (preprocess + TWO ViT-B/14 fp32 forwards at batch 1,
    place_recognition.py:759-779) on a bounded sample, find_loop_closures over N = 5000
    descriptors amortised per keyframe, and -- for the verified pairs per keyframe the
    GPU run produced -- the reference's per-pair verification cost: SuperPoint on BOTH
    images (geometric_verification.py:285-290 re-extracts per pair) + LightGlue (fp32
    restatements, oracle/), timed on one sampled pair.  RANSAC (OpenCV, C++) is not
    restated on the CPU and is excluded; it is milliseconds against seconds."""
    from oracle import lightglue as olg
    from oracle import retrieval as oret
    from oracle import superpoint as osp
    from oracle import vit as ovit
    from mlgate.weights import lightglue_state_dict, superpoint_state_dict
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(0).items()}
    rng = np.random.default_rng(0)
    n_done, t_vit, t0 = 0, 0.0, time.perf_counter()
    while n_done < 32 and (time.perf_counter() - t0) < budget_s * 0.5:
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
    sample = (f"{n_done} keyframes x (preprocess + 2 ViT-B/14 fp32 forwards, batch 1) = {t_vit:.1f} s; "
              f"find_loop_closures N=5000 D=768 k=10 = {t_knn:.2f} s, amortised per keyframe")
    if pairs_per_kf > 0:
        frames = make_frames(np.arange(2), 1, torch.device("cpu")).numpy()
        s = time.perf_counter()
        f = osp.superpoint(superpoint_state_dict(0), [frames[0], frames[1]], emulate_bf16=False)
        olg.Oracle(lightglue_state_dict(0), emulate_bf16=False).match(
            f[0]["keypoints"], f[0]["descriptors"], f[1]["keypoints"], f[1]["descriptors"])
        t_pair = time.perf_counter() - s
        per_kf += pairs_per_kf * t_pair
        sample += (f"; 1 pair x (SuperPoint on both images + LightGlue, fp32) = {t_pair:.1f} s, "
                   f"x {pairs_per_kf:.2f} gate-accepted pairs per keyframe")
    return {"value": round(1.0 / per_kf, 4), "unit": "keyframes/s", "cores": threads, "kind": "port",
            "sample": sample}


class Gate:
    """The per-rank pipeline state: frames, engines, cross-rank gathers."""

    def __init__(self, args, world, rank, dev):
        self.args, self.world, self.rank, self.dev = args, world, rank, dev
        N = self.N = args.keyframes
        self.lo, self.hi = mdist.shard(N, world, rank)
        self.n_local = self.hi - self.lo
        self.t_all = torch.from_numpy(np.arange(N) * 0.765).to(dev)
        self.f_all = torch.from_numpy(floors_for(N)).to(dev)
        self.hf_all = torch.ones(N, dtype=torch.uint8, device=dev)
        self.frames = make_frames(np.arange(self.lo, self.hi), args.places, dev)
        self.eng = VitB14(synthetic_state_dict(0), device=dev, max_batch=args.batch)
        self.gather = mdist.RowGather(N, EMBED, world, dev)
        self.desc_loc = self.gather.out[self.lo:self.hi] if world == 1 else torch.empty(self.n_local, EMBED, device=dev)
        self.local_feats = torch.empty(self.n_local, self.eng.n_local, EMBED, dtype=torch.float32, device=dev)
        self.totals = torch.zeros(2, dtype=torch.int64, device=dev)
        self.verify = args.verify == "all"
        if self.verify:
            self.sp = SuperPointGPU(device=dev, max_num_keypoints=KP)
            self.lg = LightGlueGPU(device=dev)
            self.g_kp = mdist.RowGather(N, KP * 2, world, dev)
            self.g_ds = mdist.RowGather(N, KP * 256, world, dev)
            self.g_cnt = mdist.RowGather(N, 1, world, dev, dtype=torch.int32)
            if world == 1:
                self.kp_loc, self.ds_loc = self.g_kp.out, self.g_ds.out
                self.cnt_loc = self.g_cnt.out
            else:
                self.kp_loc = torch.empty(self.n_local, KP * 2, device=dev)
                self.ds_loc = torch.empty(self.n_local, KP * 256, device=dev)
                self.cnt_loc = torch.empty(self.n_local, 1, dtype=torch.int32, device=dev)
            self.K = torch.from_numpy(ISEC_K.reshape(9).copy()).to(dev)
        self.stats = {}

    def step(self):
        a = self.args
        self.eng.forward_into(self.frames, self.desc_loc, self.local_feats)
        if self.world > 1:
            self.gather(self.desc_loc)  # RCCL all-gather of the descriptors over xGMI
        self.totals.zero_()
        idx, sim, valid, count = retrieval.knn_gate(self.gather.out, self.t_all, self.f_all, self.hf_all, 10.0, 0.5,
                                                    a.k, True, q0=self.lo, Q=self.n_local, totals=self.totals)
        if not self.verify:
            return 0, 0
        # SuperPoint once per keyframe (the reference re-extracts per pair), cached in HBM
        for b0 in range(0, self.n_local, a.sp_batch):
            b1 = min(self.n_local, b0 + a.sp_batch)
            kp, _, ds, _, cnt = self.sp.extract_device(self.frames[b0:b1])
            self.kp_loc[b0:b1].copy_(kp.view(b1 - b0, -1))
            self.ds_loc[b0:b1].copy_(ds.view(b1 - b0, -1))
            self.cnt_loc[b0:b1, 0].copy_(cnt)
        if self.world > 1:
            self.g_kp(self.kp_loc)
            self.g_ds(self.ds_loc)
            self.g_cnt(self.cnt_loc)
        kp_all = self.g_kp.out.view(self.N, KP, 2)
        ds_all = self.g_ds.out.view(self.N, KP, 256)
        counts = self.g_cnt.out.view(-1).cpu().numpy()
        # gate-accepted candidates of this rank's queries
        k = idx.shape[1]
        ok = (valid.bool() & (torch.arange(k, device=self.dev)[None, :] < count[:, None].long()))
        qs, js = torch.nonzero(ok, as_tuple=True)
        pa_t, pb_t = (qs + self.lo).to(torch.int32), idx[qs, js].to(torch.int32)
        # pair-level load balance across ranks (features are all-gathered, so any rank
        # can verify any pair; the union of the slices is the global pair list)
        pa_t, pb_t = mdist.balanced_pairs(pa_t, pb_t, self.world, self.rank)
        pa = pa_t.cpu().numpy()
        pb = pb_t.cpu().numpy()
        verified = 0
        for c0 in range(0, len(pa), a.lg_chunk):
            ca, cb = pa[c0:c0 + a.lg_chunk], pb[c0:c0 + a.lg_chunk]
            m, _, n, _ = self.lg.match_device(kp_all, ds_all, counts, ca, cb)
            # matched keypoints -> one batched RANSAC (essential matrix, K = ISEC cam1) + pose
            P = len(ca)
            live = torch.arange(KP, device=self.dev)[None, :] < n[:, None]
            pi, si = torch.nonzero(live, as_tuple=True)
            ta = torch.from_numpy(ca).to(self.dev).long()[pi]
            tb = torch.from_numpy(cb).to(self.dev).long()[pi]
            k1 = kp_all[ta, m[pi, si, 0].long()].contiguous()
            k2 = kp_all[tb, m[pi, si, 1].long()].contiguous()
            offs = torch.zeros(P + 1, dtype=torch.int32, device=self.dev)
            offs[1:] = torch.cumsum(n, 0)
            _, _, inl, _, _ = geometry.epipolar_ransac_device(k1, k2, offs, self.K, 0, 3.0)
            ratio = inl.float() / n.clamp(min=1).float()
            ok_v = (n >= 5) & (inl >= 20) & (ratio >= 0.25)
            verified += int(ok_v.sum())
        return len(pa), verified


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--keyframes", type=int, default=5000)
    # 123 frames = 65,190 tokens = 255 M-tiles of 256: the 256x256 GEMM tiles of every
    # ViT layer (3 / 9 / 12 N-tiles) then fill 256 CUs in whole waves (99.6 %).
    ap.add_argument("--batch", type=int, default=123)
    ap.add_argument("--sp-batch", type=int, default=64)
    ap.add_argument("--lg-chunk", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--places", type=int, default=600)
    ap.add_argument("--verify", choices=["all", "none"], default="all")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    gate = Gate(args, world, rank, dev)
    L = _native.lib()
    all_slots = (1 << len(SLOTS)) - 1
    for i in range(args.warmup):
        if i == args.warmup - 1:
            _native.check(L.mlg_prof_enable(all_slots), "prof")
        gate.step()
    torch.cuda.synchronize()
    tot, tflops = {}, {}
    for s in SLOTS:
        ms, cnt, work = ctypes.c_double(), ctypes.c_long(), ctypes.c_double()
        L.mlg_prof_read(s, ctypes.byref(ms), ctypes.byref(cnt))
        L.mlg_prof_read_work(s, ctypes.byref(work))
        tot[s] = ms.value
        tflops[s] = work.value / (ms.value * 1e9) if ms.value > 0 else 0.0  # TFLOP/s, or TB/s for HBM_SLOTS
    dom = max(tot, key=tot.get) if args.warmup > 0 else 0
    L.mlg_prof_reset()
    _native.check(L.mlg_prof_enable(1 << dom), "prof")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pairs = verified = 0
    for _ in range(args.steps):
        p, v = gate.step()
        pairs += p
        verified += v
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    L.mlg_prof_enable(0)
    ms, cnt, work = ctypes.c_double(), ctypes.c_long(), ctypes.c_double()
    L.mlg_prof_read(dom, ctypes.byref(ms), ctypes.byref(cnt))
    L.mlg_prof_read_work(dom, ctypes.byref(work))
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
    pv = torch.tensor([pairs, verified], dtype=torch.int64, device=dev)
    totals = gate.totals
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(totals)
        dist.all_reduce(pv)
    dt = dt_t.item()
    N = args.keyframes

    if rank == 0:
        avg_s = ms.value / 1e3 / max(cnt.value, 1)
        flops = work.value / max(cnt.value, 1)  # algorithmic FLOPs (bytes) per launch (averaged)
        hbm = dom in HBM_SLOTS
        achieved = (flops / avg_s / (1e9 if hbm else 1e12)) if cnt.value else None
        peak = HBM_PEAK_GBS if hbm else MFMA_BF16_PEAK_TFLOPS
        valid, rejected = (int(x) for x in totals.cpu())
        n_pairs, n_ver = (int(x) for x in pv.cpu())
        steps = max(args.steps, 1)
        line = {
            "metric": "keyframes gated/sec (VPR+kNN+LightGlue verify)" if gate.verify else
                      "keyframes gated/sec (CricaVPR DINOv2-B/14 descriptor + cosine-kNN floor gate)",
            "value": round(N * args.steps / dt, 2), "unit": "keyframes/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic 640x480x3 uint8 BGR keyframes (rectangle scenes, revisits, cross-floor aliasing); "
                    "seeded synthetic DINOv2-B/14, SuperPoint and LightGlue weights (no network for checkpoints)",
            "config": {"workload": "configs[1] CricaVPR (DINOv2-B/14 @322, GeM) descriptors + local features + "
                                   "all-keyframes cosine-kNN (k=%d, gap 10 s, thr 0.5) + floor gate" % args.k
                                   + ("; configs[2] SuperPoint(2048) + LightGlue + E-RANSAC/recoverPose on every "
                                      "gate-accepted candidate" if gate.verify else ""),
                       "keyframes": N, "vit_batch": args.batch, "parallelism": f"frame-sharded x{world}",
                       "gate_valid": valid, "gate_rejected": rejected,  # per step (totals of the last step)
                       "pairs_verified": n_pairs // steps, "pairs_geometrically_valid": n_ver // steps},
            "roofline": {"kernel": SLOTS[dom], "bound": "hbm" if hbm else "mfma",
                         "achieved": round(achieved, 2) if achieved else None,
                         "peak": peak, "unit": "GB/s" if hbm else "TFLOP/s",
                         "frac": round(achieved / peak, 4) if achieved else None,
                         "traffic": pmc_traffic(SLOTS[dom]), "avg_launch_us": round(avg_s * 1e6, 2),
                         "launches": cnt.value,
                         ("bytes_per_launch" if hbm else "flops_per_launch"): round(flops, 1),
                         "stage_ms_per_step": {SLOTS[s]: round(tot[s], 2) for s in SLOTS},
                         "stage_rate": {SLOTS[s]: (f"{tflops[s] * 1e3:.0f} GB/s" if s in HBM_SLOTS else
                                                   f"{tflops[s]:.1f} TFLOP/s") for s in SLOTS}},
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(pairs_per_kf=(n_pairs / steps / N) if gate.verify else 0.0)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
