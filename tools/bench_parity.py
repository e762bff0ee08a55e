"""Bench-scale parity against the fp32 chain (GPU box checker tool).

    python tools/bench_parity.py retrieval [--out gpurun_out/bench_retrieval.npz]
    python tools/bench_parity.py probe
    python tools/bench_parity.py chain [--out gpurun_out/bench_chain.npz] [--workers 16]

``retrieval``: bench.py's workload (5000 keyframes, 600 places, k = 20) through the
product's DeviceGate (bf16 ViT, fused kNN gate), and the same keyframes through the fp32
restatements -- oracle.vit (hub DINOv2-B/14 + GeM, place_recognition.py:613-643,
781-803; torch fp32, placed on the GPU only for speed) and oracle.retrieval
.find_loop_closures (:851-911, the per-row loop restated in C).  Writes both descriptor
sets and both retrieval results, and prints how many (q, m, is_valid) entries differ.

``chain``: one bench step of the product (DeviceGate, record=True) and the whole fp32
chain of SURVEY.md §3.5 on the same keyframes: fp32 descriptors -> find_loop_closures ->
verify_with_semantics on every floor-valid match (SuperPoint + LightGlue restated in fp32,
on the device; OpenCV's findEssentialMat RANSAC loop restated in C, oracle/csrc/ransac_cv.c,
on a host process pool; the decision rule of geometric_verification.py:602-620).  Every
ordered pair either side verifies gets both decisions.  Writes the fp32 chain's retrieval
(with each row's top k + 8 fp32 candidates, for near-tie margins) and per-pair results.

``probe``: times the fp32 SuperPoint / LightGlue restatements on the device and the
numpy OpenCV-RANSAC restatement on the host (sizing of the whole-step verifier check).

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
from mlgate import synthetic  # noqa: E402
from mlgate.pipeline import DeviceGate  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402


def _fp32_only():
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False


def log(**kw):
    print(json.dumps(kw), flush=True)


def oracle_descriptors(frames, sd, dev, batch=32):
    """fp32 CricaVPR descriptors of device uint8 frames [N, H, W, 3] via oracle.vit."""
    from oracle import vit as ovit
    osd = {k: torch.from_numpy(np.asarray(v)).to(dev) for k, v in sd.items()}
    n = frames.shape[0]
    X = np.empty((n, 768), np.float32)
    t0 = time.time()
    for b0 in range(0, n, batch):
        b1 = min(n, b0 + batch)
        fr = frames[b0:b1].cpu().numpy()
        x = torch.cat([ovit.preprocess(f) for f in fr]).to(dev)
        X[b0:b1] = ovit.gem(ovit.forward_tokens(x, osd)).cpu().numpy()
        if b0 % 1024 == 0:
            log(phase="fp32_vit", done=b1, s=round(time.time() - t0, 1))
    return X


def retrieval(a):
    from oracle import pipeline as opipe
    from oracle import retrieval as oret
    _fp32_only()
    dev = torch.device("cuda:0")
    N, k = a.keyframes, a.k
    seq, labels = bench.sequence(N, a.places)
    frames = synthetic.frames_device(seq, np.arange(N), dev)
    sd = synthetic_state_dict(0)
    gate = DeviceGate(frames, seq.t, labels, 1, 0, dev, k=k, verify=False, vit_batch=246, vit_state_dict=sd,
                      record=True)
    gate.step()
    torch.cuda.synchronize()
    X_gpu = gate.gather.out.cpu().numpy().copy()
    idx, sim, valid, count = gate.last_retrieval
    del gate
    torch.cuda.empty_cache()
    log(phase="device_gate", matches=int(count.sum()))
    X32 = oracle_descriptors(frames, sd, dev)
    codes, has = opipe.floor_codes(labels)
    q32, m32, s32, v32 = oret.find_loop_closures(X32, seq.t, codes, has, 10.0, 0.5, k, True)
    sel = np.arange(idx.shape[1])[None, :] < count[:, None]
    qg, mg, sg, vg = np.repeat(np.arange(N), count), idx[sel].astype(np.int64), sim[sel], valid[sel].astype(bool)
    cos = np.sum(X_gpu.astype(np.float64) * X32, 1) / (np.linalg.norm(X_gpu.astype(np.float64), axis=1)
                                                       * np.linalg.norm(X32.astype(np.float64), axis=1))
    tg = set(zip(qg.tolist(), mg.tolist(), vg.tolist()))
    t32 = set(zip(q32.tolist(), m32.tolist(), np.asarray(v32, bool).tolist()))
    rows_differ = len({q for q, _, _ in tg ^ t32})
    rep = {"keyframes": N, "k": k, "matches_gpu": len(qg), "matches_fp32": len(q32),
           "triples_only_gpu": len(tg - t32), "triples_only_fp32": len(t32 - tg), "rows_differ": rows_differ,
           "floor_rejected_gpu": int((~vg).sum()), "floor_rejected_fp32": int((~np.asarray(v32, bool)).sum()),
           "ordered_lists_equal": bool(len(qg) == len(q32) and np.array_equal(mg, m32)),
           "desc_1mcos_max": float(1 - cos.min()), "desc_1mcos_median": float(np.median(1 - cos)),
           "sim_absdiff_max_on_common": None}
    common = {(q, m) for q, m, _ in tg} & {(q, m) for q, m, _ in t32}
    if common:
        dg = {(q, m): s for q, m, s in zip(qg.tolist(), mg.tolist(), sg.tolist())}
        d32 = {(q, m): s for q, m, s in zip(q32.tolist(), m32.tolist(), np.asarray(s32).tolist())}
        rep["sim_absdiff_max_on_common"] = float(max(abs(dg[c] - d32[c]) for c in common))
    log(**rep)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.savez_compressed(a.out, X_gpu=X_gpu, X32=X32, idx=idx, sim=sim, valid=valid, count=count, q32=q32, m32=m32,
                        s32=s32, v32=np.asarray(v32, np.uint8), labels=np.asarray(labels), t=seq.t,
                        report=json.dumps(rep))


def probe(a):
    from mlgate.weights import lightglue_state_dict, superpoint_state_dict
    from oracle import geometry as ogeo
    from oracle import lightglue as olg
    from oracle import superpoint as osp
    _fp32_only()
    dev = torch.device("cuda:0")
    seq, _ = bench.sequence(a.keyframes, a.places)
    po = seq.place_of
    pairs = [(i, j) for i in range(400) for j in range(i + 14, 400) if po[i] >= 0 and po[i] == po[j]][:24]
    used = sorted({x for p in pairs for x in p})
    imgs = synthetic.frames_host(seq, used)
    spsd = superpoint_state_dict(0)
    feats = []
    for rep in range(2):  # the second pass is timed (MIOpen finds its kernels per shape on the first)
        torch.cuda.synchronize()
        t0 = time.time()
        feats = []
        for b0 in range(0, len(used) - len(used) % 8, 8):
            feats += osp.superpoint(spsd, imgs[b0:b0 + 8], emulate_bf16=False, device=dev)
        torch.cuda.synchronize()
        t_sp = (time.time() - t0) / len(feats)
        log(phase="sp", rep=rep, ms_per_frame=round(t_sp * 1e3, 2))
    used = used[:len(feats)]
    pairs = [(p, q) for p, q in pairs if p in used and q in used]
    fi = {f: feats[i] for i, f in enumerate(used)}
    lg = olg.Oracle(lightglue_state_dict(0), emulate_bf16=False, device=dev)
    lg.match(fi[pairs[0][0]]["keypoints"], fi[pairs[0][0]]["descriptors"], fi[pairs[0][1]]["keypoints"],
             fi[pairs[0][1]]["descriptors"])
    torch.cuda.synchronize()
    t0 = time.time()
    res = []
    for p, q in pairs:
        r = lg.match(fi[p]["keypoints"], fi[p]["descriptors"], fi[q]["keypoints"], fi[q]["descriptors"])
        res.append((p, q, r["matches"].cpu().numpy(), r["stop"]))
    torch.cuda.synchronize()
    t_lg = (time.time() - t0) / len(pairs)
    t0 = time.time()
    inl = []
    for p, q, mm, _ in res[:4]:
        k1 = fi[p]["keypoints"].cpu().numpy()[mm[:, 0]]
        k2 = fi[q]["keypoints"].cpu().numpy()[mm[:, 1]]
        inl.append(int(ogeo.cv_ransac(k1, k2, ogeo.ISEC_K, 3.0)[2]) if len(mm) >= 5 else 0)
    t_rs = (time.time() - t0) / 4
    log(sp_ms_per_frame=round(t_sp * 1e3, 2), lg_ms_per_pair=round(t_lg * 1e3, 2),
        ransac_py_s_per_pair=round(t_rs, 2), keypoints=[int(len(fi[u]["keypoints"])) for u in used[:4]],
        matches=[int(len(r[2])) for r in res[:8]], stops=[r[3] for r in res[:8]], inliers=inl)


def _ransac_job(job):
    """(key, k1, k2) -> (key, inliers, packed mask, model or None) with the C twin of
    findEssentialMat (pool worker)."""
    from oracle import _lib
    from oracle import geometry as ogeo
    key, k1, k2 = job
    M, mask, g = _lib.essential_ransac(k1, k2, ogeo.ISEC_K, 3.0)
    return key, g, np.packbits(mask), (None if M is None else np.asarray(M, np.float64).reshape(3, 3))


def _capture_product_ransac(store):
    """Wrap mlgate.geometry.epipolar_ransac_device so every RANSAC call of the product gate
    also leaves its inputs and outputs (host copies) in `store`: the product's own match
    lists, for the GPU-vs-C-twin check on identical lists."""
    from mlgate import geometry as mgeo
    orig = mgeo.epipolar_ransac_device

    def hook(k1, k2, offs, K=None, k_stride=0, threshold=3.0, **kw):
        out = orig(k1, k2, offs, K, k_stride, threshold, **kw)
        o = offs.cpu().numpy()  # on the current (RANSAC side) stream: ordered after the launch
        store.append((k1[:int(o[-1])].cpu().numpy(), k2[:int(o[-1])].cpu().numpy(), o, out[2].cpu().numpy(),
                      out[1][:int(o[-1])].cpu().numpy(), out[0].cpu().numpy(), out[4].cpu().numpy()))
        return out
    mgeo.epipolar_ransac_device = hook
    return orig


def _same_model(gpu_model, twin_model):
    """the GPU's model (None when it found none) vs the twin's, bit for bit"""
    if gpu_model is None or twin_model is None:
        return gpu_model is None and twin_model is None
    return np.array_equal(np.asarray(gpu_model, np.float64).reshape(3, 3).view(np.uint64),
                          np.asarray(twin_model, np.float64).reshape(3, 3).view(np.uint64))


def _twin_report(pool, lists, gpu_inl, gpu_masks, gpu_models, label):
    """GPU RANSAC vs the C twin on the same lists: counts, masks and model bits, pair by pair."""
    jobs = [pool.apply_async(_ransac_job, ((i, k1, k2),)) for i, (k1, k2) in enumerate(lists)]
    eq_n = eq_m = eq_e = 0
    bad = []
    for job in jobs:
        i, g, pm, M = job.get()
        same_n = int(gpu_inl[i]) == int(g)
        same_m = np.array_equal(np.packbits(gpu_masks[i].astype(bool)), pm)
        same_e = _same_model(gpu_models[i], M)
        eq_n += same_n
        eq_m += same_m
        eq_e += same_e
        if not (same_n and same_m and same_e) and len(bad) < 20:
            bad.append({"pair": i, "matches": len(lists[i][0]), "gpu": int(gpu_inl[i]), "twin": int(g),
                        "model_equal": bool(same_e)})
    n = max(len(lists), 1)
    rep = {"check": label, "pairs": len(lists), "inliers_equal_c_twin": eq_n / n, "masks_equal_c_twin": eq_m / n,
           "models_equal_c_twin": eq_e / n, "differ": bad}
    log(**rep)
    return rep


def chain(a):
    import multiprocessing as mp
    pool = mp.get_context("fork").Pool(a.workers)  # forked before the process touches the GPU
    from mlgate.weights import lightglue_state_dict, superpoint_state_dict
    from oracle import lightglue as olg
    from oracle import pipeline as opipe
    from oracle import retrieval as oret
    from oracle import superpoint as osp
    _fp32_only()
    t0 = time.time()
    dev = torch.device("cuda:0")
    N, k = a.keyframes, a.k
    seq, labels = bench.sequence(N, a.places)
    labels = np.asarray(labels)
    frames = synthetic.frames_device(seq, np.arange(N), dev)
    sd = synthetic_state_dict(0)
    gate = DeviceGate(frames, seq.t, labels, 1, 0, dev, k=k, verify=True, K=bench.ISEC_K, vit_batch=246, sp_batch=64,
                      lg_chunk=a.lg_chunk, vit_state_dict=sd, record=True)
    captured = []
    orig_ransac = _capture_product_ransac(captured)
    counts_gpu = gate.step()
    torch.cuda.synchronize()
    from mlgate import geometry as mgeo
    mgeo.epipolar_ransac_device = orig_ransac
    # (1) the product's own match lists: its GPU RANSAC vs the C twin, every ordered pair
    p_lists, p_inl, p_masks, p_models = [], [], [], []
    for k1c, k2c, o, inl_c, mask_c, model_c, status_c in captured:
        for p_ in range(len(o) - 1):
            p_lists.append((k1c[o[p_]:o[p_ + 1]], k2c[o[p_]:o[p_ + 1]]))
            p_inl.append(inl_c[p_])
            p_masks.append(mask_c[o[p_]:o[p_ + 1]])
            p_models.append(None if int(status_c[p_]) == 1 else model_c[p_])
    del captured
    twin_product = _twin_report(pool, p_lists, p_inl, p_masks, p_models, "product lists: GPU RANSAC vs C twin")
    del p_lists, p_inl, p_masks, p_models
    gr = gate.last_pair_results
    g_idx, g_sim, g_valid, g_count = gate.last_retrieval
    del gate
    torch.cuda.empty_cache()
    log(phase="device_gate", s=round(time.time() - t0, 1), **counts_gpu)
    X32 = oracle_descriptors(frames, sd, dev)
    codes, has = opipe.floor_codes(labels)
    q32, m32, s32, v32 = oret.find_loop_closures(X32, seq.t, codes, has, 10.0, 0.5, k, True)
    v32 = np.asarray(v32, bool)
    # each row's top k + 8 fp32 candidates after the time mask (near-tie margins of the test)
    Xn = torch.from_numpy(oret.normalize_rows(X32)).to(dev)
    tt = torch.from_numpy(seq.t).to(dev)
    ext_i = np.zeros((N, k + 8), np.int16)
    ext_s = np.zeros((N, k + 8), np.float32)
    for r0 in range(0, N, 1000):
        S = Xn[r0:r0 + 1000] @ Xn.T
        S[(tt[r0:r0 + 1000, None] - tt[None, :]).abs() < 10.0] = -float("inf")
        v, i = torch.topk(S, k + 8, dim=1)
        ext_i[r0:r0 + 1000], ext_s[r0:r0 + 1000] = i.cpu().numpy(), v.cpu().numpy()
    # verify_with_semantics on every is_valid match (its floor check never skips them:
    # gated retrieval already required equal floors)
    fp_pairs = [(int(q), int(m)) for q, m, v in zip(q32, m32, v32) if v and labels[q] == labels[m]]
    gpu_pairs = list(zip(gr["a"].tolist(), gr["b"].tolist()))
    union = sorted(set(fp_pairs) | set(gpu_pairs))
    log(phase="fp32_retrieval", s=round(time.time() - t0, 1), matches=len(q32), floor_rejected=int((~v32).sum()),
        fp32_pairs=len(fp_pairs), gpu_pairs=len(gpu_pairs), union=len(union))
    used = sorted({f for p in union for f in p})
    spsd = superpoint_state_dict(0)
    feats = {}
    for b0 in range(0, len(used), 8):
        idx = used[b0:b0 + 8]
        imgs = frames[torch.as_tensor(idx, device=dev)].cpu().numpy()
        for f, ft in zip(idx, osp.superpoint(spsd, imgs, emulate_bf16=False, device=dev)):
            feats[f] = (ft["keypoints"], ft["descriptors"], ft["keypoints"].cpu().numpy())
    log(phase="fp32_superpoint", s=round(time.time() - t0, 1), frames=len(used))
    lg = olg.Oracle(lightglue_state_dict(0), emulate_bf16=False, device=dev)
    nm = np.zeros(len(union), np.int32)
    stop = np.zeros(len(union), np.int8)
    pending, f_lists = [], []
    for i, (p, q) in enumerate(union):
        r = lg.match(feats[p][0], feats[p][1], feats[q][0], feats[q][1])
        mm = r["matches"].cpu().numpy()
        nm[i], stop[i] = len(mm), r["stop"]
        f_lists.append((feats[p][2][mm[:, 0]], feats[q][2][mm[:, 1]]))
        pending.append(pool.apply_async(_ransac_job, ((i,) + f_lists[-1],)))
        if i % 2000 == 0:
            log(phase="fp32_lightglue", done=i, s=round(time.time() - t0, 1))
    inl = np.zeros(len(union), np.int32)
    f_masks = [None] * len(union)
    f_models = [None] * len(union)
    for job in pending:
        i, g, pm, M = job.get()
        inl[i] = g
        f_masks[i] = pm
        f_models[i] = M
    # (2) the fp32 chain's lists through the product's GPU RANSAC (batched as the gate
    # calls it) against the C twin's counts / masks just computed
    from mlgate import geometry as mgeo
    g_inl = np.zeros(len(union), np.int32)
    g_eq_m = g_eq_e = 0
    for c0 in range(0, len(union), 4096):
        rs = mgeo.epipolar_ransac([x[0] for x in f_lists[c0:c0 + 4096]], [x[1] for x in f_lists[c0:c0 + 4096]],
                                  bench.ISEC_K, 3.0, device=str(dev))
        for j, r in enumerate(rs):
            g_inl[c0 + j] = r.inliers
            g_eq_m += np.array_equal(np.packbits(r.mask), f_masks[c0 + j])
            g_eq_e += _same_model(r.model, f_models[c0 + j])
    twin_fp32 = {"check": "fp32 chain lists: GPU RANSAC vs C twin", "pairs": len(union),
                 "inliers_equal_c_twin": float((g_inl == inl).mean()) if len(union) else 1.0,
                 "masks_equal_c_twin": g_eq_m / max(len(union), 1),
                 "models_equal_c_twin": g_eq_e / max(len(union), 1),
                 "differ": [{"pair": int(i), "matches": int(nm[i]), "gpu": int(g_inl[i]), "twin": int(inl[i])}
                            for i in np.flatnonzero(g_inl != inl)[:20]]}
    log(**twin_fp32)
    del f_lists, f_masks, f_models
    pool.close()
    ratio = inl / np.maximum(nm, 1)
    fvalid = (nm >= 5) & (inl >= 20) & (ratio >= 0.25)
    gi = {pq: j for j, pq in enumerate(gpu_pairs)}
    in_gpu = np.array([pq in gi for pq in union])
    fset = set(fp_pairs)
    in_fp = np.array([pq in fset for pq in union])
    gm = np.full(len(union), -1, np.int32)
    gin = np.full(len(union), -1, np.int32)
    gv = np.zeros(len(union), bool)
    for i, pq in enumerate(union):
        j = gi.get(pq)
        if j is not None:
            gm[i], gin[i], gv[i] = gr["matches"][j], gr["inliers"][j], gr["is_valid"][j]
    both = in_gpu & in_fp
    flips = np.flatnonzero(both & (gv != fvalid))
    counts_fp = {"retrieval_floor_rejected": int((~v32).sum()), "skipped_floor_mismatch": 0,
                 "verifier_invalid": int(len(fp_pairs) - (fvalid & in_fp).sum()), "gate_rejected_cross_floor": 0}
    counts_fp["total"] = sum(counts_fp.values())
    rep = {"keyframes": N, "k": k, "pairs_fp32": len(fp_pairs), "pairs_gpu": len(gpu_pairs),
           "pairs_common": int(both.sum()), "fp32_valid": int((fvalid & in_fp).sum()),
           "gpu_valid": int(gv[in_gpu].sum()), "decision_flips_on_common": len(flips),
           "flips": [{"a": union[i][0], "b": union[i][1], "gpu": [int(gm[i]), int(gin[i]), bool(gv[i])],
                      "fp32": [int(nm[i]), int(inl[i]), bool(fvalid[i])]} for i in flips[:50]],
           "counts_fp32": counts_fp, "counts_gpu": counts_gpu, "twin_product": twin_product, "twin_fp32": twin_fp32,
           "s": round(time.time() - t0, 1)}
    log(**rep)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.savez_compressed(a.out, keyframes=N, places=a.places, k=k, labels=labels, count32=np.bincount(q32, minlength=N)
                        .astype(np.int16), m32=m32.astype(np.int16), s32=np.asarray(s32, np.float32),
                        v32=v32, ext_i=ext_i, ext_s=ext_s, a=np.array([p for p, _ in union], np.int16),
                        b=np.array([q for _, q in union], np.int16), in_gpu=in_gpu, in_fp32=in_fp,
                        fp32_matches=nm.astype(np.int16), fp32_inliers=inl.astype(np.int16), fp32_is_valid=fvalid,
                        fp32_stop=stop, gpu_matches=gm.astype(np.int16), gpu_inliers=gin.astype(np.int16),
                        gpu_is_valid=gv, report=json.dumps(rep))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("phase", choices=["retrieval", "probe", "chain"])
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--lg-chunk", type=int, default=5120)
    ap.add_argument("--keyframes", type=int, default=5000)
    ap.add_argument("--places", type=int, default=600)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/bench_retrieval.npz")
    a = ap.parse_args()
    {"retrieval": retrieval, "probe": probe, "chain": chain}[a.phase](a)


if __name__ == "__main__":
    main()
