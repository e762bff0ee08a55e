"""Where do the product's SuperPoint + LightGlue matches leave the fp32 chain, and how far
do two fp32 realisations of the reference chain leave each other?  (GPU box tool; VERDICT
r04 "next 1": the fp32 noise floor of bench-scale decisions and a per-site probe.)

Sample: the ordered pairs of tests/golden/bench_chain_fp32.npz that both chains verified
-- every pair whose fp32 inlier ratio lies within 0.04 of the 0.25 threshold ("near") and
a seeded sample of the others.  The keyframes are bench.py's (5000, 600 places).

Each CHAIN is (SuperPoint realisation, LightGlue realisation) followed by the same RANSAC
(findEssentialMat, K = ISEC cam1, threshold 3 px: the product's mlg_ransac_epipolar, which
replays OpenCV's sample stream; its inlier counts on the fp32 lists are checked against the
fixture's C-twin counts, oracle/csrc/ransac_cv.c) and the decision rule
(geometric_verification.py:602-620).  Realisations:
  SuperPoint  hip      the product (csrc/superpoint.hip)
              f32      oracle.superpoint in fp32 (on the device)
              f32perm  the same with every conv's input channels in a seeded permuted order
              f64      float64
              tf32     conv inputs / weights rounded to TF32: cuDNN's default on Ampere+
                       (torch.backends.cudnn.allow_tf32 = True), the reference's SuperPoint on CUDA
              bf16w / bf16act / bf16   bf16 weights / stored activations / both (the kernels' sites)
  LightGlue   hip      the product (csrc/lightglue.hip + lg_proj / attention / lg_ffn)
              f32, f32perm, f64        as above (oracle.lightglue)
              fp16attn the reference's CUDA attention: SDPA on x.half() (FlashAttention)
              bf16:<site> / bf16all    bf16 operands at one product site / all of them
Every chain is compared with (f32, f32): match list identical, match count identical,
|d matches|, |d inliers| and decision flips, over all sampled pairs and over "near".
Two RANSAC-only controls on the (f32, f32) lists: the same matches in a seeded shuffled
order (4 seeds; OpenCV's fixed cv::RNG stream then draws other samples -- a fresh RANSAC
draw on the same match set), and one match dropped (4 seeded choices) -- the decision's
sensitivity to the sample stream alone and to a one-match change.

    python tools/lg_precision_probe.py --set floor [--pairs 2000]
    python tools/lg_precision_probe.py --set sites [--pairs 1000]

Writes one JSON line per chain (stdout) and gpurun_out/lgp_<set>.npz (per-pair counts).
Test infrastructure: the oracle is the checker here, never the thing measured."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-level-indoor-slam_amd")]

import bench  # noqa: E402
from mlgate import geometry, synthetic  # noqa: E402
from mlgate.lightglue import LightGlueGPU  # noqa: E402
from mlgate.superpoint import SuperPointGPU  # noqa: E402
from mlgate.weights import lightglue_state_dict, superpoint_state_dict  # noqa: E402
from oracle import lightglue as olg  # noqa: E402
from oracle import superpoint as osp  # noqa: E402

KP = 2048
SETS = {
    "floor": [("f32", "f32"), ("hip", "hip"), ("f32", "hip"), ("hip", "f32"), ("f32perm", "f32perm"),
              ("f64", "f64"), ("tf32", "fp16attn"), ("f32", "fp16attn"), ("tf32", "f32")],
    "sites": [("f32", "f32")] + [("f32", f"bf16:{s}") for s in olg.SITES] + [("f32", "bf16all"), ("bf16w", "f32"),
                                                                              ("bf16act", "f32"), ("bf16", "f32")],
}


def log(**kw):
    print(json.dumps(kw), flush=True)


def sample_pairs(fx, n_rand, seed=0):
    both = fx["in_gpu"] & fx["in_fp32"]
    ratio = fx["fp32_inliers"] / np.maximum(fx["fp32_matches"].astype(np.float64), 1)
    near = np.flatnonzero(both & (np.abs(ratio - 0.25) <= 0.04))
    rest = np.flatnonzero(both & ~(np.abs(ratio - 0.25) <= 0.04))
    pick = np.random.default_rng(seed).choice(rest, min(n_rand, len(rest)), replace=False)
    sel = np.concatenate([near, np.sort(pick)])
    return sel, len(near)


def sp_realisation(name, frames_dev, used, sd, dev):
    """-> (kp [F, KP, 2], desc [F, KP, 256], counts [F] host): device tensors (f32, or f64 for f64)."""
    F_ = len(used)
    if name == "hip":
        sp = SuperPointGPU(state_dict=sd, device=dev, max_num_keypoints=KP)
        kp = torch.zeros(F_, KP, 2, device=dev)
        ds = torch.zeros(F_, KP, 256, device=dev)
        cnt = np.zeros(F_, np.int64)
        for b0 in range(0, F_, 64):
            fr = frames_dev[torch.as_tensor(used[b0:b0 + 64], device=dev)]
            k, _, d, _, c = sp.extract_device(fr)
            kp[b0:b0 + len(fr)], ds[b0:b0 + len(fr)] = k, d
            cnt[b0:b0 + len(fr)] = c.cpu().numpy()
        return kp, ds, cnt
    kw = {"f32": {}, "f32perm": {"perm_seed": 1}, "f64": {"dtype": torch.float64}, "tf32": {"tf32": True},
          "bf16w": {"sites": ("w",)}, "bf16act": {"sites": ("act",)}, "bf16": {"sites": ("w", "act")}}[name]
    dt = kw.get("dtype", torch.float32)
    kp = torch.zeros(F_, KP, 2, device=dev, dtype=dt)
    ds = torch.zeros(F_, KP, 256, device=dev, dtype=dt)
    cnt = np.zeros(F_, np.int64)
    bs = 4 if dt == torch.float64 else 8
    for b0 in range(0, F_, bs):
        imgs = frames_dev[torch.as_tensor(used[b0:b0 + bs], device=dev)].cpu().numpy()
        for j, ft in enumerate(osp.superpoint(sd, imgs, emulate_bf16=False, device=dev, **kw)):
            n = len(ft["keypoints"])
            kp[b0 + j, :n], ds[b0 + j, :n], cnt[b0 + j] = ft["keypoints"], ft["descriptors"], n
    return kp, ds, cnt


def lg_oracle(name, sd, dev):
    if name == "f32":
        return olg.Oracle(sd, emulate_bf16=False, device=dev)
    if name == "f32perm":
        return olg.Oracle(sd, emulate_bf16=False, device=dev, perm_seed=1)
    if name == "f64":
        return olg.Oracle(sd, emulate_bf16=False, device=dev, dtype=torch.float64)
    if name == "fp16attn":
        return olg.Oracle(sd, emulate_bf16=False, device=dev, attn_fp16=True)
    if name == "bf16all":
        return olg.Oracle(sd, emulate_bf16=True, device=dev)
    if name.startswith("bf16:"):
        return olg.Oracle(sd, emulate_bf16=False, device=dev, sites=(name[5:],))
    raise KeyError(name)


def lg_realisation(name, feats, ia, ib, sd, dev):
    """-> list of int64 [n, 2] match arrays (indices into each image's keypoints)."""
    kp, ds, cnt = feats
    if name == "hip":
        lg = LightGlueGPU(state_dict=sd, device=dev)
        out = []
        kp32, ds32 = kp.float().contiguous(), ds.float().contiguous()
        for c0 in range(0, len(ia), 1024):
            m, _, n, _ = lg.match_device(kp32, ds32, cnt, ia[c0:c0 + 1024], ib[c0:c0 + 1024])
            m, n = m.cpu().numpy(), n.cpu().numpy()
            out += [m[i, :n[i]].astype(np.int64) for i in range(len(n))]
        return out
    lg = lg_oracle(name, sd, dev)
    out = []
    for a, b in zip(ia, ib):
        r = lg.match(kp[a, :cnt[a]], ds[a, :cnt[a]], kp[b, :cnt[b]], ds[b, :cnt[b]])
        out.append(r["matches"].cpu().numpy().astype(np.int64))
    return out


def ransac(feats, ia, ib, matches, dev):
    """Inlier counts of findEssentialMat on each pair's matched keypoints (pixels, f32)."""
    kp = feats[0].float()
    k1, k2, offs = [], [], [0]
    for a, b, m in zip(ia, ib, matches):
        mt = torch.as_tensor(m, device=dev)
        k1.append(kp[a][mt[:, 0]] if len(m) else kp.new_zeros(0, 2))
        k2.append(kp[b][mt[:, 1]] if len(m) else kp.new_zeros(0, 2))
        offs.append(offs[-1] + len(m))
    K = torch.from_numpy(bench.ISEC_K.reshape(9).copy()).to(dev)
    offs_t = torch.as_tensor(offs, dtype=torch.int32, device=dev)
    _, _, inl, _, _ = geometry.epipolar_ransac_device(torch.cat(k1).contiguous(), torch.cat(k2).contiguous(), offs_t,
                                                      K, 0, 3.0, with_pose=False)
    return inl.cpu().numpy().astype(np.int64)


def _c_twin(job):
    """(i, k1, k2) -> (i, inliers) with oracle/csrc/ransac_cv.c (pool worker)."""
    from oracle import _lib
    from oracle import geometry as ogeo
    i, k1, k2 = job
    return i, (_lib.essential_ransac(k1, k2, ogeo.ISEC_K, 3.0)[2] if len(k1) >= 5 else 0)


def decide(n, inl):
    return (n >= 5) & (inl >= 20) & (inl / np.maximum(n, 1) >= 0.25)


def coords(feats, ia, ib, lists):
    """Matched keypoint coordinates [n, 4] (x0, y0, x1, y1) per pair: what RANSAC consumes, in
    its order (keypoint indices are not comparable across SuperPoint realisations: a score
    change reorders the top-k)."""
    kp = feats[0].float().cpu().numpy()
    return [np.concatenate([kp[a][m[:, 0]], kp[b][m[:, 1]]], 1) if len(m) else np.zeros((0, 4), np.float32)
            for a, b, m in zip(ia, ib, lists)]


def compare(name, base, other, n_near):
    """Statistics of chain `other` against `base` (dicts: xy, n, inl, ok): the match list
    identical as RANSAC sees it (same coordinates in the same order), as a set, counts."""
    same_list = np.array([x.shape == y.shape and np.array_equal(x, y) for x, y in zip(base["xy"], other["xy"])])
    same_set = np.array([x.shape == y.shape and set(map(tuple, x.tolist())) == set(map(tuple, y.tolist()))
                         for x, y in zip(base["xy"], other["xy"])])
    dn = np.abs(other["n"] - base["n"])
    di = np.abs(other["inl"] - base["inl"])
    flip = other["ok"] != base["ok"]
    rel = di / np.maximum(base["inl"], 1)
    q = lambda a, p: float(np.percentile(a, p)) if len(a) else None  # noqa: E731
    return {"chain": name, "pairs": len(dn), "near": n_near, "list_identical": float(same_list.mean()),
            "set_identical": float(same_set.mean()),
            "count_identical": float((dn == 0).mean()), "dmatches_median": q(dn, 50), "dmatches_p99": q(dn, 99),
            "dinliers_median": q(di, 50), "dinliers_p99": q(di, 99), "dinliers_max": int(di.max()),
            "rel_dinliers_p90": q(rel, 90), "rel_dinliers_p99": q(rel, 99),
            "flips": int(flip.sum()), "flips_near": int(flip[:n_near].sum()),
            "flips_far": int(flip[n_near:].sum()),
            "list_identical_near": float(same_list[:n_near].mean()) if n_near else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", choices=sorted(SETS), default="floor")
    ap.add_argument("--pairs", type=int, default=2000)
    ap.add_argument("--chains", default="", help="comma list of sp/lg to run instead of the set")
    ap.add_argument("--out", default="gpurun_out")
    ap.add_argument("--c-twin", default="", help="comma list of chains whose lists also go through the C twin "
                                                   "of findEssentialMat (oracle/csrc/ransac_cv.c) on a host pool")
    ap.add_argument("--save-xy", default="", help="comma list of chains whose match coordinates are saved")
    ap.add_argument("--workers", type=int, default=16)
    a = ap.parse_args()
    pool = None
    if a.c_twin:
        import multiprocessing as mp
        pool = mp.get_context("fork").Pool(a.workers)  # forked before the process touches the GPU
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    dev = torch.device("cuda:0")
    t0 = time.time()
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "bench_chain_fp32.npz")))
    sel, n_near = sample_pairs(fx, a.pairs)
    pa, pb = fx["a"][sel].astype(np.int64), fx["b"][sel].astype(np.int64)
    used = np.unique(np.concatenate([pa, pb]))
    ia, ib = np.searchsorted(used, pa), np.searchsorted(used, pb)
    log(phase="sample", pairs=len(sel), near=n_near, frames=len(used))
    N, places = int(fx["keyframes"]), int(fx["places"])
    seq, _ = bench.sequence(N, places)
    frames = synthetic.frames_device(seq, np.arange(N), dev)
    chains = SETS[a.set] if not a.chains else [tuple(c.split("/")) for c in a.chains.split(",")]
    spsd, lgsd = superpoint_state_dict(0), lightglue_state_dict(0)
    feats, res, rows = {}, {}, []
    for sp_name, lg_name in chains:
        if sp_name not in feats:
            feats[sp_name] = sp_realisation(sp_name, frames, used, spsd, dev)
            log(phase="superpoint", name=sp_name, s=round(time.time() - t0, 1))
        lists = lg_realisation(lg_name, feats[sp_name], ia, ib, lgsd, dev)
        n = np.array([len(m) for m in lists], np.int64)
        inl = ransac(feats[sp_name], ia, ib, lists, dev)
        key = f"{sp_name}/{lg_name}"
        xy = coords(feats[sp_name], ia, ib, lists)
        res[key] = {"xy": xy, "n": n, "inl": inl, "ok": decide(n, inl)}
        log(phase="chain", name=key, s=round(time.time() - t0, 1))
        if key == "f32/f32":  # the fixture's fp32 chain: same lists -> the C twin's inlier counts
            rep = {"chain": "f32/f32 vs fixture", "matches_equal": float((n == fx["fp32_matches"][sel]).mean()),
                   "inliers_equal_c_twin": float((inl == fx["fp32_inliers"][sel]).mean()),
                   "decisions_equal": float((res[key]["ok"] == fx["fp32_is_valid"][sel]).mean())}
            log(**rep)
            rows.append(rep)
            base = res[key]
            for s in (1, 2, 3, 4):  # RANSAC-only controls on the fp32 lists
                rng = np.random.default_rng(s)
                sh = [m[rng.permutation(len(m))] for m in lists]
                inl_s = ransac(feats[sp_name], ia, ib, sh, dev)
                r = compare(f"f32/f32 shuffled ({s})", base, {"xy": coords(feats[sp_name], ia, ib, sh), "n": n, "inl": inl_s,
                                                               "ok": decide(n, inl_s)}, n_near)
                log(**r)
                rows.append(r)
            for s in (1, 2, 3, 4):
                rng = np.random.default_rng(100 + s)
                dl = [np.delete(m, rng.integers(0, len(m)), axis=0) if len(m) > 5 else m for m in lists]
                n_d = np.array([len(m) for m in dl], np.int64)
                inl_d = ransac(feats[sp_name], ia, ib, dl, dev)
                r = compare(f"f32/f32 one match dropped ({s})", base, {"xy": coords(feats[sp_name], ia, ib, dl), "n": n_d,
                                                                       "inl": inl_d,
                                                                       "ok": decide(n_d, inl_d)}, n_near)
                log(**r)
                rows.append(r)
        elif key == "hip/hip":
            rep = {"chain": "hip/hip vs fixture product", "matches_equal": float((n == fx["gpu_matches"][sel]).mean()),
                   "inliers_equal": float((inl == fx["gpu_inliers"][sel]).mean())}
            log(**rep)
            rows.append(rep)
        if "f32/f32" in res and key != "f32/f32":
            r = compare(key, res["f32/f32"], res[key], n_near)
            log(**r)
            rows.append(r)
    if "f64/f64" in res and "f32/f32" in res:
        for key in ("f32/f32", "hip/hip", "f32perm/f32perm", "tf32/fp16attn"):
            if key in res:
                r = compare(f"{key} vs f64/f64", res["f64/f64"], res[key], n_near)
                log(**r)
                rows.append(r)
    if "hip/hip" in res and "tf32/fp16attn" in res:
        r = compare("hip/hip vs tf32/fp16attn", res["tf32/fp16attn"], res["hip/hip"], n_near)
        log(**r)
        rows.append(r)
    xy_out = {}
    for key in [c for c in a.save_xy.split(",") if c in res]:
        xy = res[key]["xy"]
        xy_out[f"{key}|xy"] = np.concatenate(xy).astype(np.float32)
        xy_out[f"{key}|offs"] = np.concatenate([[0], np.cumsum([len(x) for x in xy])]).astype(np.int64)
    for key in [c for c in a.c_twin.split(",") if c in res]:
        # the same lists through the C twin: GPU RANSAC == OpenCV's loop restated, pair by pair
        jobs = [pool.apply_async(_c_twin, ((i, x[:, :2], x[:, 2:]),)) for i, x in enumerate(res[key]["xy"])]
        inl_c = np.zeros(len(jobs), np.int64)
        for j in jobs:
            i, g = j.get()
            inl_c[i] = g
        eq = inl_c == res[key]["inl"]
        r = {"chain": f"{key}: GPU RANSAC vs C twin on the same lists", "inliers_equal": float(eq.mean()),
             "differ": [(int(i), int(res[key]["inl"][i]), int(inl_c[i]), int(res[key]["n"][i]))
                        for i in np.flatnonzero(~eq)[:20]]}
        log(**r)
        rows.append(r)
        xy_out[f"{key}|inl_c"] = inl_c
    os.makedirs(a.out, exist_ok=True)
    np.savez_compressed(os.path.join(a.out, f"lgp_{a.set}.npz"), a=pa, b=pb, near=n_near,
                        **{f"{k}|{f}": v[f] for k, v in res.items() for f in ("n", "inl", "ok")},
                        report=json.dumps(rows), **xy_out)
    log(phase="done", s=round(time.time() - t0, 1))


if __name__ == "__main__":
    main()
