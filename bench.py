"""Benchmark: the full semantic loop-closure gate (BASELINE configs[3])
over a 5k-keyframe multi-floor sequence on 1..8 MI355X (BASELINE.json metric
"keyframes gated/sec (VPR+kNN+LightGlue verify)").

The floor labels come from IMUFloorDetector on the sequence's 200 Hz IMU log (host, once,
before the timed region: they are an input of the gate, kilobytes per sequence).  One
step = the whole sequence gated once (mlgate.pipeline.DeviceGate): every keyframe
(640x480x3 uint8 BGR, resident in HBM) preprocessed and run through ViT-B/14 (the
split-bf16 forward by default, --vit; one forward yields the GeM descriptor and the
cached local features, as CricaVPR.add_image needs); all keyframes
retrieved against all (top-k = 20 as configs[2], time gap, threshold, floor decision);
every floor-valid candidate verified (verify_with_semantics): SuperPoint keypoints /
descriptors per keyframe (computed once, cached), LightGlue on the pair, OpenCV-sequenced
essential-matrix RANSAC + recoverPose with K = ISEC cam1, the verifier's decision rule
(>= 20 inliers, ratio >= 0.25); the floor gate on the geometrically valid pairs.  The
line reports the four-term false-loop-closure rejection count of the step.
Multi-GPU: frames are sharded across ranks (strong scaling: fixed total); descriptors
are all-gathered over RCCL; each rank gates its own query rows, the gate-accepted pairs
are all-gathered and re-split evenly (unordered pairs kept on one rank) for verification,
and each rank receives the SuperPoint features of exactly the keyframes its pairs touch
(all_to_all); the counts are all-reduced.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--verify all|none]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import re
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
sys.path.insert(0, ROOT)

from mlgate import _native, synthetic  # noqa: E402
from mlgate import distributed as mdist  # noqa: E402
from mlgate.pipeline import DeviceGate, floor_labels_from_imu  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md, no sparsity)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
SLOTS = {0: "vit_fc1_gemm", 1: "vit_fc2_gemm", 2: "vit_qkv_gemm", 3: "vit_proj_gemm", 4: "vit_attention",
         5: "lightglue_attention", 6: "lightglue_qkv_gemms", 7: "superpoint_conv3x3", 8: "lightglue_ffn_fused"}
# slots whose recorded work is algorithmic HBM bytes (bound "hbm"), not FLOPs: none since
# the fused FFN (slot 8, 256 FLOP per HBM byte, at the ridge) is priced in FLOPs
HBM_SLOTS = set()
VIT_SLOTS = {0, 1, 2, 3, 4}  # ViT GEMMs + attention (split forward: 3 MFMA products per product)
ISEC_K = np.array([[893.63, 0.0, 376.95], [0.0, 893.97, 266.57], [0.0, 0.0, 1.0]])  # cam1, SURVEY §8


def sequence(n, places, seed=0):
    """The synthetic ISEC-shaped sequence (mlgate.synthetic): keyframe times, the IMU
    log and the floor labels IMUFloorDetector assigns from it (floor_detector.py:63-156)."""
    seq = synthetic.make_sequence(n, places, seed)
    labels, _ = floor_labels_from_imu(seq.t, synthetic.imu_log(seq), start_floor=5)
    return seq, labels


def pmc_traffic(slot_name, lg_chunk):
    """HBM bytes per launch of the dominant kernel from the committed PMC pass
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from separate
    `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` runs of one LightGlue call of this
    bench's size, with the gfx950 FETCH_SIZE x2 correction of MI355X_MICROARCH.md), or None
    if absent or measured on a call of another size than --lg-chunk."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        entry = json.load(f).get(slot_name)
    if not entry:
        return None
    pairs = entry.get("pairs")
    if pairs is None:
        m = re.search(r"--pairs (\d+)", entry.get("source", ""))
        pairs = int(m.group(1)) if m else None
    return entry.get("bytes_per_launch") if pairs == lg_chunk else None


def host_threads():
    """Threads for the CPU legs: the CPUs this process may use.  BASELINE.md asks for
    os.cpu_count(); on the GPU box that reports the whole machine while the job's share is
    16 CPUs (OMP_NUM_THREADS=16 is exported there), and threads beyond the share only
    oversubscribe it -- so the share, when the environment states it."""
    env = os.environ.get("OMP_NUM_THREADS")
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(int(env), avail)) if env and env.isdigit() else avail


def cpu_baseline(budget_s=12.0, pairs_per_kf=0.0):
    """The oracle port of the reference CPU path on this host's cores, per keyframe:
    CricaVPR.add_image (preprocess + TWO ViT-B/14 fp32 forwards at batch 1,
    place_recognition.py:759-779) on a bounded sample, find_loop_closures over N = 5000
    descriptors amortised per keyframe, and -- for the verified pairs per keyframe the
    GPU run produced -- the reference's per-pair verification cost: SuperPoint on BOTH
    images (geometric_verification.py:285-290 re-extracts per pair) + LightGlue (fp32
    restatements, oracle/) + findEssentialMat's RANSAC loop (the C twin,
    oracle/csrc/ransac_cv.c) on the pair's matches, timed pair by pair on up to six pairs (one
    non-revisit, then revisits of distinct places) within the budget; their mean is the
    per-pair cost and their spread is reported.  Plus configs[0]:
    MixVPR's ResNet-50 fallback (place_recognition.py:248-306) + find_loop_closures on 64
    keyframes, the reference's CPU plumbing configuration."""
    from oracle import _lib as olib
    from oracle import geometry as ogeo
    from oracle import lightglue as olg
    from oracle import resnet as orn
    from oracle import retrieval as oret
    from oracle import superpoint as osp
    from oracle import vit as ovit
    from mlgate.weights import lightglue_state_dict, resnet50_state_dict, superpoint_state_dict
    threads = host_threads()
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
    X = rng.standard_normal((n, 768)).astype(np.float32)
    t = np.arange(n) * 0.765
    labels = sequence(n, 600)[1]
    s = time.perf_counter()
    oret.find_loop_closures(X, t, labels, np.ones(n, np.uint8), 10.0, 0.5, 20, True)
    t_knn_c = time.perf_counter() - s
    # the reference's own per-row Python loop (place_recognition.py:872-909) on a bounded
    # set of query rows, extrapolated to all N rows (every row costs the same O(N) mask +
    # argsort); np.dot for the similarity matrix as the reference builds it
    s = time.perf_counter()
    S = oret.pairwise_similarities(X)
    t_dot = time.perf_counter() - s
    rows = 250
    s = time.perf_counter()
    oret.find_loop_closures_loop(X, t, list(labels), 10.0, 0.5, 20, True, rows=range(rows), S=S)
    t_knn = t_dot + (time.perf_counter() - s) * n / rows
    per_kf = t_vit / n_done + t_knn / n
    sample = (f"{n_done} keyframes x (preprocess + 2 ViT-B/14 fp32 forwards, batch 1) = {t_vit:.1f} s; "
              f"find_loop_closures N=5000 D=768 k=20 through the reference's per-row Python loop = {t_knn:.1f} s "
              f"(np.dot {t_dot:.2f} s + {rows} of {n} rows timed, extrapolated; the C restatement of the same loop, "
              f"oracle/csrc/oracle.c, takes {t_knn_c:.2f} s), amortised per keyframe")
    if pairs_per_kf > 0:
        # verified pairs of the bench's own kind: revisits of distinct places (LightGlue's 9
        # layers, ~400 matches) and one non-revisit (early stop), each timed alone; the mean
        # is the per-pair cost, the spread is reported with it
        seq2 = synthetic.make_sequence(64, 8, 0)
        po = seq2.place_of
        pairs = [(0, next(i for i in range(64) if po[i] != po[0]))]  # the non-revisit first
        for p in range(8):
            same = [i for i in range(64) if po[i] == p]
            if len(same) >= 2:
                pairs.append((same[0], same[-1]))
            if len(pairs) == 6:
                break
        frames = synthetic.frames_host(seq2, sorted({i for pq in pairs for i in pq}))
        fidx = {f: k for k, f in enumerate(sorted({i for pq in pairs for i in pq}))}
        spsd, lgo = superpoint_state_dict(0), olg.Oracle(lightglue_state_dict(0), emulate_bf16=False)
        t_pairs = []
        for a, b in pairs:
            if (time.perf_counter() - t0) > budget_s * 2.5 and len(t_pairs) >= 2:
                break
            s = time.perf_counter()
            f = osp.superpoint(spsd, [frames[fidx[a]], frames[fidx[b]]], emulate_bf16=False)
            r = lgo.match(f[0]["keypoints"], f[0]["descriptors"], f[1]["keypoints"], f[1]["descriptors"])
            mm = r["matches"].numpy()
            olib.essential_ransac(f[0]["keypoints"].numpy()[mm[:, 0]], f[1]["keypoints"].numpy()[mm[:, 1]],
                                  ogeo.ISEC_K, 3.0)
            t_pairs.append(time.perf_counter() - s)
        t_pair = float(np.mean(t_pairs))
        per_kf += pairs_per_kf * t_pair
        sample += (f"; {len(t_pairs)} pairs (1 non-revisit + {len(t_pairs) - 1} revisits) x (SuperPoint on both "
                   f"images + LightGlue, fp32, + RANSAC) = {t_pair:.2f} s mean (min {min(t_pairs):.2f}, "
                   f"max {max(t_pairs):.2f}), x {pairs_per_kf:.2f} verified pairs per keyframe")
    # configs[0]: MixVPR ResNet-50 fallback descriptors + find_loop_closures, 64 keyframes
    seq0, lab0 = sequence(64, 16)
    fr0 = synthetic.frames_host(seq0)
    rsd = resnet50_state_dict(0)
    s = time.perf_counter()
    n0 = 0
    D0 = np.zeros((64, 4096), np.float32)
    while n0 < 64 and (time.perf_counter() - s) < budget_s * 0.5:
        D0[n0] = orn.extract_descriptor(rsd, fr0[n0])
        n0 += 1
    t_rn = time.perf_counter() - s
    s = time.perf_counter()
    oret.find_loop_closures(D0, seq0.t, lab0, np.ones(64, np.uint8), 10.0, 0.5, 10, True)
    t_k0 = time.perf_counter() - s
    c0 = {"value": round(64.0 / (t_rn / n0 * 64 + t_k0), 3), "unit": "keyframes/s",
          "sample": f"{n0} of 64 keyframes through the ResNet-50 fallback (fp32) = {t_rn:.1f} s + "
                    f"find_loop_closures over 64 x 4096 = {t_k0 * 1e3:.1f} ms"}
    return {"value": round(1.0 / per_kf, 4), "unit": "keyframes/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "sample": sample, "configs0": c0}


def configs0_bench(frames, seq, labels, lo, dev, iters=5):
    """configs[0] on the GPU: MixVPR's ResNet-50 fallback descriptors (4096-dim, zero-padded,
    place_recognition.py:248-306; HIP mlg_resnet50) of 64 keyframes and find_loop_closures
    over them (k = 10, gap 10 s, thr 0.5, floor-gated), HIP-event timed."""
    from mlgate import retrieval
    from mlgate.resnet import ResNet50GPU
    n = min(64, frames.shape[0])
    fr = frames[:n].contiguous()
    eng = ResNet50GPU(device=dev)
    t = torch.as_tensor(seq.t[lo:lo + n], device=dev)
    fl = torch.as_tensor(np.asarray(labels[lo:lo + n], np.int64), device=dev)
    hf = torch.ones(n, dtype=torch.uint8, device=dev)

    def one():
        d = eng.forward_device(fr, 4096)
        return retrieval.knn_gate(d, t, fl, hf, 10.0, 0.5, 10, True)
    one()
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        out = one()
    ev[1].record()
    torch.cuda.synchronize(dev)
    ms = ev[0].elapsed_time(ev[1]) / iters
    tf = 8.2e9 * n / (ms * 1e-3) / 1e12  # ResNet-50 @224^2 ~8.2 GFLOP per frame
    return {"workload": "configs[0] MixVPR ResNet-50 fallback descriptors (4096-dim) + find_loop_closures, "
                        "64 keyframes (seeded synthetic ResNet-50 weights)",
            "keyframes": n, "ms": round(ms, 3), "keyframes_per_s": round(n / (ms * 1e-3), 1),
            "resnet_tflops": round(tf, 1), "matches": int(out[3].sum())}


def ingest_bench(dev, n_files=1024, distinct=64):
    """Row f2: keyframe ingestion throughput.  `distinct` synthetic bench
    keyframes are written as bag_utils.extract_images writes them (scripts/utils/
    bag_utils.py:222-271: '{t:.6f}.png', bgr8 through cv2.imwrite, whose PNG default is
    zlib level 1) -- here with Pillow at compress_level 1 -- and mlgate.ingest.KeyframeStream
    (the loader process_image_sequence uses, place_recognition.py:936-991) streams n_files
    paths over them into HBM (host decode pool -> pinned buffer -> side-stream upload).
    Files repeat, so they are read from the page cache: the number is decode + upload."""
    import shutil
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    from PIL import Image
    from mlgate import ingest
    threads = host_threads()
    d = tempfile.mkdtemp(prefix="mlg_ingest_")
    try:
        seq = synthetic.make_sequence(distinct, 16, 3)
        fr = synthetic.frames_host(seq)
        names = [os.path.join(d, f"{t:.6f}.png") for t in seq.t]

        def enc(i):
            Image.fromarray(np.ascontiguousarray(fr[i][..., ::-1])).save(names[i], compress_level=1)
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(enc, range(distinct)))
        paths = [names[i % distinct] for i in range(n_files)]
        stream = ingest.KeyframeStream(paths, device=dev, batch=128, threads=threads)
        for _ in stream:  # warm-up pass (page cache, pinned buffers)
            break
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        n = 0
        for idx, frames in stream:
            n += len(idx)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        size = float(np.mean([os.path.getsize(x) for x in names]))
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return {"workload": "f2 keyframe ingestion: 640x480 bgr8 PNG keyframes (zlib level 1, bag_utils format) -> "
                        "uint8 frames in HBM via mlgate.ingest.KeyframeStream (host inflate + unfilter pool, "
                        "pinned buffer, side-stream upload)",
            "keyframes": n, "seconds": round(dt, 3), "ingest_kf_per_s": round(n / dt, 1), "threads": threads,
            "host_cpus": os.cpu_count(), "png_bytes_mean": round(size), "distinct_files": distinct,
            "source": "page cache (files repeat)"}


def _all_reduce(t, op=dist.ReduceOp.SUM):
    """in-place all-reduce of a device tensor; through the host under gloo (the one-GPU
    rehearsal, MLGATE_BENCH_REHEARSE), straight on the device under RCCL"""
    if dist.get_backend() == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)
    return t


def _lf_layer_flops(d):
    """one LoFTR encoder layer per token: q / k / v, merge, MLP 2d -> 2d -> d, the linear
    attention's KV and apply (8 heads x (d / 8)^2)"""
    return 2 * (4 * d * d + 2 * d * 2 * d + 2 * d * d + 2 * 8 * (d // 8) ** 2)


def loftr_flops_per_pair(L=4800, matches=0.0, self0_sides=2.0):
    """FLOPs of LoFTR's matching for one pair at L coarse cells (640x480: 80 x 60): 8 coarse
    encoder layers (4 self + 4 cross) on both sides, the coarse similarity L x L x 256, and
    per coarse match the fine stage (2 layers over 2 x 25 window tokens at d 128, 8 heads x
    16 x 16).  self0_sides: the pair sides layer 0 runs on -- 2 as the reference computes
    it; the product runs that self layer once per distinct frame of a call (round 6), so
    the kernel sub-run passes distinct frames / pairs and the rate counts the work done."""
    return ((7 * 2 + self0_sides) * L * _lf_layer_flops(256) + 2 * L * L * 256
            + matches * 2 * 2 * 25 * _lf_layer_flops(128))


# algorithmic FLOPs per 640x480 keyframe of LoFTR's ResNetFPN_8_2 backbone (196-channel
# stages counted at 196; the GPU runs them zero-padded to 256)
def loftr_backbone_flops(H=480, W=640):
    p2, p4, p8 = (H // 2) * (W // 2), (H // 4) * (W // 4), (H // 8) * (W // 8)
    c = [p2 * 49 * 128, 4 * p2 * 9 * 128 * 128,                                   # stem, layer1
         p4 * 9 * (128 * 196 + 3 * 196 * 196) + p4 * 128 * 196,                   # layer2
         p8 * 9 * (196 * 256 + 3 * 256 * 256) + p8 * 196 * 256,                   # layer3
         p8 * 256 * 256, p4 * (196 * 256 + 9 * 256 * 256 + 9 * 256 * 196),       # FPN 1/8, 1/4
         p2 * (128 * 196 + 9 * 196 * 196 + 9 * 196 * 128)]                       # FPN 1/2
    return 2.0 * sum(c)


def loftr_bench(frames, seq, labels, lo, dev, world, rank, n_pairs=1024, chunk=128, kernel_pairs=256):
    """configs[4]: GeometricVerifier('loftr') as the gate's matcher, batched across the ranks.
    (1) gate level -- DeviceGate(matcher='loftr') verifies the first n_pairs floor-valid
    candidate pairs of the sequence (the same kNN as the main gate), the pairs split over
    the ranks (balanced_pairs) and each rank receiving the raw frames its pairs touch;
    pairs/s = n_pairs / the slowest rank's verification time (backbone per keyframe +
    coarse / fine matching + RANSAC + decision, HIP work synchronised).  (2) kernel level,
    rank 0 -- LoFTRGPU on `kernel_pairs` revisit pairs of its shard, HIP-event timed:
    backbone and matching rates against the bf16 peak."""
    from mlgate.loftr import LoFTRGPU
    g = DeviceGate(frames, seq.t, labels, world, rank, dev, k=20, verify=True, K=ISEC_K, vit_batch=246,
                   matcher="loftr", loftr_chunk=chunk, max_pairs=n_pairs, vit_state_dict=synthetic_state_dict(0))
    g.time_verify = True
    g.step()  # warm-up
    out = g.step()
    vt = torch.tensor([g.last_verify_s], dtype=torch.float64, device=dev)
    cnt = torch.tensor([out["pairs_verified"], out["verified_valid"]], dtype=torch.int64, device=dev)
    if world > 1:
        _all_reduce(vt, dist.ReduceOp.MAX)
        _all_reduce(cnt)
    del g
    torch.cuda.empty_cache()
    res = {"workload": "configs[4] LoFTR 640x480 (seeded synthetic weights) as the gate's matcher: "
                       "ResNetFPN_8_2 backbone per keyframe + coarse linear-attention transformer, dual-softmax "
                       "mutual-NN, 5x5 fine refinement + E-RANSAC + decision per ordered pair, pairs split over "
                       f"{world} rank(s)",
           "gate_pairs": int(cnt[0]), "gate_valid": int(cnt[1]), "gate_verify_s": round(float(vt), 3),
           "gate_pairs_per_s": round(int(cnt[0]) / float(vt), 1)}
    if rank != 0:
        return res
    n = frames.shape[0]
    po = seq.place_of[lo:lo + n]
    pairs = [(i, j) for i in range(n) for j in range(i + 1, n) if po[i] >= 0 and po[i] == po[j]][:kernel_pairs]
    if not pairs:
        return res
    used = sorted({i for p in pairs for i in p})
    lf = LoFTRGPU(device=dev, feature_batch=16)
    res.update(_loftr_kernels(lf, frames[torch.as_tensor(used, device=dev)].contiguous(), used, pairs, chunk, dev))
    # the ISEC camera's own frame size (720 x 540 -> cv2 resize to 720 x 536: L = 6030
    # cells, L % 4 != 0), the same scenes rendered at that size
    isec = torch.from_numpy(synthetic.frames_host(seq, np.asarray(used) + lo, 540, 720)).to(dev)
    res["isec_720x540"] = _loftr_kernels(lf, isec, used, pairs, chunk, dev)
    return res


def _loftr_kernels(lf, sel, used, pairs, chunk, dev):
    """LoFTRGPU backbone + matching of `pairs` (indices into `used`, the frames of `sel`),
    HIP-event timed after a warm-up pass, with their algorithmic rates."""
    pos = {f: k for k, f in enumerate(used)}
    pa, pb = [pos[a] for a, _ in pairs], [pos[b] for _, b in pairs]
    H, W = int(sel.shape[1]) // 8 * 8, int(sel.shape[2]) // 8 * 8

    def match_all(coarse, fine):
        ms = []
        for c0 in range(0, len(pairs), chunk):
            c, *_ = lf.match_device(coarse, fine, H, W, pa[c0:c0 + chunk], pb[c0:c0 + chunk])
            ms.append(c)
        return torch.cat(ms)
    coarse, fine = lf.features(sel)
    cntm = match_all(coarse, fine)
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    coarse, fine = lf.features(sel)
    ev[1].record()
    cntm = match_all(coarse, fine)
    ev[2].record()
    torch.cuda.synchronize(dev)
    t_feat, t_match = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
    m = float(cntm.float().mean())
    # layer 0 runs once per distinct frame of each match_device call
    nu = sum(len(set(pa[c0:c0 + chunk]) | set(pb[c0:c0 + chunk])) for c0 in range(0, len(pairs), chunk))
    bf, mf = loftr_backbone_flops(H, W), loftr_flops_per_pair((H // 8) * (W // 8), m, nu / max(len(pairs), 1))
    bt = bf * len(used) / (t_feat * 1e-3) / 1e12
    mt = mf * len(pairs) / (t_match * 1e-3) / 1e12
    return {"frame": f"{int(sel.shape[2])}x{int(sel.shape[1])} (network {W}x{H}, L = {(H // 8) * (W // 8)})",
            "kernel_keyframes": len(used), "kernel_pairs": len(pairs), "matches_mean": round(m, 1),
            "backbone_ms_per_keyframe": round(t_feat / len(used), 3), "backbone_tflops": round(bt, 1),
            "backbone_frac": round(bt / MFMA_BF16_PEAK_TFLOPS, 4),
            "match_ms_per_pair": round(t_match / len(pairs), 3), "match_tflops": round(mt, 1),
            "match_frac": round(mt / MFMA_BF16_PEAK_TFLOPS, 4),
            "flops": {"backbone_per_keyframe": bf, "match_per_pair": round(mf, 0),
                      "layer0_sides_per_pair": round(nu / max(len(pairs), 1), 3)}}


def stress_bench(n, k, dev):
    """SURVEY §8d's stress size: the same gate over an n-keyframe sequence (places scaled as
    bench.py's 600 per 5000) on one GPU, the LightGlue chunk sized from the free HBM and the
    local-feature cache (31 GB at 19,163) unmaterialised; one warm-up step, one timed step."""
    seq, labels = sequence(n, max(1, round(n * 600 / 5000)))
    frames = synthetic.frames_device(seq, np.arange(n), dev)
    g = DeviceGate(frames, seq.t, labels, 1, 0, dev, k=k, verify=True, K=ISEC_K, vit_batch=246, lg_chunk="auto",
                   local_features=False, vit_state_dict=synthetic_state_dict(0))
    g.step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    c = g.step()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    rej = c["retrieval_floor_rejected"] + c["skipped_floor_mismatch"] + c["verifier_invalid"] + \
        c["gate_rejected_cross_floor"]
    out = {"workload": f"configs[3] gate over {n} keyframes (ORB-SLAM3 pose count of the ISEC run, SURVEY §8d), "
                       "lg_chunk auto, local features not materialised",
           "keyframes": n, "seconds": round(dt, 3), "keyframes_per_s": round(n / dt, 1),
           "lg_chunk": g.last_lg_chunk, "pairs_verified": c["pairs_verified"], "verified_valid": c["verified_valid"],
           "false_loop_closure_rejections": rej,
           "peak_hbm_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1)}
    del g, frames
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--keyframes", type=int, default=5000)
    # 246 frames = 130,380 tokens = 510 M-tiles of 256: the 256x256 GEMM tiles of every
    # ViT layer (3 / 9 / 12 N-tiles) then fill 256 CUs in whole waves (99.6 %); against 123
    # frames (255 M-tiles) the ViT stages take 700 vs 728 ms per step on one box
    # (profiles/r03aw_vit_batch_sweep.txt)
    ap.add_argument("--batch", type=int, default=246)
    ap.add_argument("--sp-batch", type=int, default=64)
    # pairs per LightGlue call: 4096 (131 GB of workspace) measured 547 vs 529 kf/s at 1024
    # (profiles/r02t_chunk_sweep.txt); 5120 (164 GB, 5 calls per step instead of 6) another
    # +0.3-0.5 % and 6144 (196 GB) no more (profiles/r03as_chunk_sweep.txt); 8192 would need 260 GB
    ap.add_argument("--lg-chunk", type=int, default=5120)
    ap.add_argument("--lg-tail", type=int, default=0,
                    help="last LightGlue chunk = 1/N of the remainder (its RANSAC runs alone); 0 = off "
                         "(same-box A/B: no gain, profiles/r04p_ab_lg_tail.txt)")
    ap.add_argument("--k", type=int, default=20)  # configs[2]: top-20 candidates per query
    ap.add_argument("--places", type=int, default=600)
    ap.add_argument("--verify", choices=["all", "none"], default="all")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ingest", action="store_true", help="skip the f2 ingestion sub-object")
    ap.add_argument("--loftr-pairs", type=int, default=1024, help="configs[4] LoFTR sub-object: gate pairs (0: skip)")
    ap.add_argument("--stress-keyframes", type=int, default=0,
                    help="also gate an N-keyframe sequence once warm (SURVEY §8d: 19163, the ORB-SLAM3 pose count) "
                         "on one GPU and report it as the 'stress' sub-object (0: skip; one rank only)")
    ap.add_argument("--vit", choices=["split", "bf16"], default="split",
                    help="split: split-bf16 ViT (MLG_VIT_SPLIT, fp32-faithful descriptors); bf16: plain bf16 operands")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MLGATE_BENCH_REHEARSE=1: every rank on cuda:0 over gloo -- a one-GPU rehearsal of the
    # multi-rank bench flow (collectives, per-rank line, sub-benches); its timing means nothing
    rehearse = os.environ.get("MLGATE_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    seq, labels = sequence(args.keyframes, args.places)
    lo, hi = mdist.shard(args.keyframes, world, rank)
    frames = synthetic.frames_device(seq, np.arange(lo, hi), dev)
    gate = DeviceGate(frames, seq.t, labels, world, rank, dev, k=args.k, verify=args.verify == "all", K=ISEC_K,
                      vit_batch=args.batch, sp_batch=args.sp_batch, lg_chunk=args.lg_chunk, lg_tail=args.lg_tail,
                      vit_state_dict=synthetic_state_dict(0), vit_precise=args.vit == "split")
    ops = _native.ops()  # torch.ops.mlgate (HIP-event profiling slots of the C ABI)
    all_slots = (1 << len(SLOTS)) - 1
    for i in range(args.warmup):
        if i == args.warmup - 1:
            _native.check(ops.prof_enable(all_slots), "prof")
        gate.step()
    torch.cuda.synchronize()
    tot, tflops = {}, {}
    for s in SLOTS:
        ms, _, work = ops.prof_read(s)
        tot[s] = ms
        tflops[s] = work / (ms * 1e9) if ms > 0 else 0.0  # TFLOP/s, or TB/s for HBM_SLOTS
    dom = max(tot, key=tot.get) if args.warmup > 0 else 0
    ops.prof_reset()
    _native.check(ops.prof_enable(1 << dom), "prof")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    counts = {}
    for _ in range(args.steps):
        for key, v in gate.step().items():
            counts[key] = counts.get(key, 0) + v
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ops.prof_enable(0)
    ms, cnt, work = ops.prof_read(dom)
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
    keys = sorted(counts)
    cv = torch.tensor([counts[k_] for k_ in keys], dtype=torch.int64, device=dev)
    per_rank = None
    if world > 1:
        # per-rank view (the slowest rank sets the step): this rank's wall time, its share
        # of the verification pairs and its profiled warmup step's stage times
        mine = torch.tensor([dt / max(args.steps, 1) * 1e3, counts.get("pairs_verified", 0) / max(args.steps, 1),
                             counts.get("pairs_matched_lightglue", 0) / max(args.steps, 1)]
                            + [tot[s_] for s_ in SLOTS], dtype=torch.float64, device=dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        mdist.all_gather_into(allr, mine)
        per_rank = [{"rank": r_, "ms_per_step": round(float(v[0]), 1), "pairs_verified": int(v[1]),
                     "pairs_matched_lightglue": int(v[2]),
                     "stage_ms_warmup_step": {SLOTS[s_]: round(float(v[3 + s_]), 1) for s_ in SLOTS}}
                    for r_, v in enumerate(x.cpu().numpy() for x in allr)]
        _all_reduce(dt_t, dist.ReduceOp.MAX)
        _all_reduce(cv)
    dt = dt_t.item()
    steps = max(args.steps, 1)
    counts = {k_: int(v) // steps for k_, v in zip(keys, cv.cpu().tolist())}  # per step, all ranks
    N = args.keyframes
    torch.cuda.empty_cache()  # the main gate's LightGlue workspace
    lft = loftr_bench(frames, seq, labels, lo, dev, world, rank, args.loftr_pairs) if args.loftr_pairs > 0 else None
    c0 = configs0_bench(frames, seq, labels, lo, dev) if rank == 0 else None
    ing = ingest_bench(dev) if rank == 0 and not args.no_ingest else None
    stress = None
    if args.stress_keyframes > 0 and world == 1:
        del gate, frames
        torch.cuda.empty_cache()
        stress = stress_bench(args.stress_keyframes, args.k, dev)

    if rank == 0:
        avg_s = ms / 1e3 / max(cnt, 1)
        flops = work / max(cnt, 1)  # algorithmic FLOPs (bytes) per launch (averaged)
        hbm = dom in HBM_SLOTS
        achieved = (flops / avg_s / (1e9 if hbm else 1e12)) if cnt else None
        peak = HBM_PEAK_GBS if hbm else MFMA_BF16_PEAK_TFLOPS
        rej = {k_: counts[k_] for k_ in ("retrieval_floor_rejected", "skipped_floor_mismatch", "verifier_invalid",
                                          "gate_rejected_cross_floor")}
        rej["total"] = sum(rej.values())
        line = {
            "metric": "keyframes gated/sec (VPR+kNN+LightGlue verify)" if args.verify == "all" else
                      "keyframes gated/sec (CricaVPR DINOv2-B/14 descriptor + cosine-kNN floor gate)",
            "value": round(N * args.steps / dt, 2), "unit": "keyframes/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic 640x480x3 uint8 BGR keyframes (mlgate.synthetic: rectangle-scene places revisited "
                    "with 8-px shifts, aliased across floors; 200 Hz IMU with elevator rides -> IMUFloorDetector "
                    "labels); seeded synthetic DINOv2-B/14, SuperPoint (whitened descriptor head) and LightGlue "
                    "weights (no network for checkpoints)",
            "config": {"workload": "configs[3] full semantic gate: IMU floor labels + configs[1] CricaVPR "
                                   "(DINOv2-B/14 @322, GeM) descriptors + local features + all-keyframes cosine-kNN "
                                   "(k=%d, gap 10 s, thr 0.5) + floor-gated retrieval" % args.k
                                   + ("; configs[2] verify_with_semantics on every floor-valid candidate: "
                                      "SuperPoint(2048) + LightGlue + OpenCV-sequenced E-RANSAC (K = ISEC cam1) + "
                                      "decision rule (LightGlue once per unordered pair, RANSAC + decision per ordered pair); "
                                      "floor gate on the geometrically valid pairs"
                                      if args.verify == "all" else ""),
                       "keyframes": N, "k": args.k, "vit_batch": args.batch, "parallelism": f"frame-sharded x{world}",
                       "matches": counts["matches"], "pairs_verified": counts["pairs_verified"],
                       "pairs_matched_lightglue": counts.get("pairs_matched_lightglue", 0),
                       "pairs_geometrically_valid": counts["verified_valid"],
                       "loop_closures_accepted": counts["accepted"],
                       "superpoint_features_exchanged_gb": round(counts.get("features_exchanged_bytes", 0) / 1e9, 3),
                       "false_loop_closure_rejections": rej},
            "roofline": {"kernel": SLOTS[dom], "bound": "hbm" if hbm else "mfma",
                         "achieved": round(achieved, 2) if achieved else None,
                         "peak": peak, "unit": "GB/s" if hbm else "TFLOP/s",
                         "frac": round(achieved / peak, 4) if achieved else None,
                         "traffic": pmc_traffic(SLOTS[dom], args.lg_chunk), "avg_launch_us": round(avg_s * 1e6, 2),
                         "launches": cnt,
                         ("bytes_per_launch" if hbm else "flops_per_launch"): round(flops, 1),
                         "stage_ms_per_step": {SLOTS[s]: round(tot[s], 2) for s in SLOTS},
                         "stage_rate": {SLOTS[s]: (f"{tflops[s] * 1e3:.0f} GB/s" if s in HBM_SLOTS else
                                                   f"{tflops[s]:.1f} TFLOP/s") for s in SLOTS},
                         # the split-bf16 ViT runs 3 MFMA products per algorithmic product
                         # (hi*hi + lo*hi + hi*lo): stage_rate counts the MFMA work it issues,
                         # stage_rate_algorithmic the network's own FLOPs (2 M N K per GEMM)
                         "stage_rate_algorithmic": {
                             SLOTS[s]: f"{tflops[s] / (3.0 if args.vit == 'split' and s in VIT_SLOTS else 1.0):.1f} TFLOP/s"
                             for s in SLOTS if s not in HBM_SLOTS},
                         "vit_mfma_products_per_flop": 3 if args.vit == "split" else 1},
        }
        if per_rank:
            line["per_rank"] = per_rank
        if lft:
            line["loftr"] = lft
        if c0:
            line["configs0"] = c0
        if ing:
            line["ingest"] = ing
        if stress:
            line["stress"] = stress
        if not args.no_cpu_baseline:
            # rank 0 only, after the timed region (at world > 1 the other ranks wait at the
            # final barrier, so their processes leave the host cores to it)
            line["cpu_baseline"] = cpu_baseline(pairs_per_kf=(counts["pairs_verified"] / N) if args.verify == "all" else 0.0)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
