"""fp32 cross-check of bench-scale verifier decisions (CPU, this container; VERDICT r02
item 3).  Input: tools/decision_sample.py's npz (GPU per-pair results on a seeded sample
of one bench step's verified ordered pairs).  For every sampled pair it regenerates the
two keyframes (mlgate.synthetic.frames_host: same seeds as the GPU run) and runs the fp32
chain -- oracle.pipeline.verify_pair: SuperPoint and LightGlue without bf16 emulation,
OpenCV's RANSAC loop restated (oracle.geometry.cv_ransac), the decision rule of
geometric_verification.py:602-620 -- then reports how often the GPU decision differs.

    python tools/decision_check_cpu.py gpurun_out/decision_sample.npz [--out tests/golden/decision_sample.npz]
"""
import argparse
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-level-indoor-slam_amd")]

_W = {}


def _init(n, places, seed):
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)
    import torch
    torch.set_num_threads(1)
    from mlgate import synthetic
    from mlgate.weights import lightglue_state_dict, superpoint_state_dict
    from oracle import pipeline as opipe
    _W["seq"] = synthetic.make_sequence(n, places, seed)
    _W["sp"] = superpoint_state_dict(0)
    _W["lg"] = opipe.make_matcher(lightglue_state_dict(0))


def _feats(i):
    from mlgate import synthetic
    from oracle import superpoint as osp
    if i not in _W:
        img = synthetic.frames_host(_W["seq"], [i])[0]
        _W[i] = osp.superpoint(_W["sp"], [img], emulate_bf16=False)[0]
    return _W[i]


def _verify(pair):
    from oracle import geometry as ogeo
    from oracle import pipeline as opipe
    a, b = pair
    r = opipe.verify_pair(None, None, _W["sp"], _W["lg"], ogeo.ISEC_K, feats=(_feats(a), _feats(b)))
    r.pop("matches")
    return pair, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sample")
    ap.add_argument("--out", default=None)
    ap.add_argument("--workers", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    g = dict(np.load(a.sample))
    pairs = [(int(x), int(y)) for x, y in zip(g["a"], g["b"])]
    # group pairs sharing a frame into one worker's chunk as far as order allows (feature cache)
    t0 = time.time()
    with Pool(a.workers, initializer=_init, initargs=(int(g["keyframes"]), int(g["places"]), int(g["seq_seed"]))) as p:
        res = dict(p.map(_verify, pairs, chunksize=4))
    ref_valid = np.array([res[q]["is_valid"] for q in pairs])
    ref_n = np.array([res[q]["num_matches"] for q in pairs])
    ref_in = np.array([res[q]["num_inliers"] for q in pairs])
    ref_stop = np.array([res[q]["stop"] for q in pairs])
    gv = g["is_valid"].astype(bool)
    flips = np.nonzero(gv != ref_valid)[0]
    both = gv & ref_valid
    rel_in = np.abs(g["inliers"][both] - ref_in[both]) / np.maximum(ref_in[both], 1)
    rel_n = np.abs(g["matches"] - ref_n) / np.maximum(ref_n, 1)
    report = {"pairs": len(pairs), "gpu_valid": int(gv.sum()), "fp32_valid": int(ref_valid.sum()),
              "decision_flips": int(len(flips)), "flip_rate": round(len(flips) / max(len(pairs), 1), 5),
              "flipped_pairs": [{"a": pairs[i][0], "b": pairs[i][1], "gpu": [int(g["matches"][i]), int(g["inliers"][i]),
                                                                          bool(gv[i])],
                                 "fp32": [int(ref_n[i]), int(ref_in[i]), bool(ref_valid[i])]} for i in flips[:20]],
              "matches_rel_diff_median": round(float(np.median(rel_n)), 4),
              "matches_rel_diff_p99": round(float(np.quantile(rel_n, 0.99)), 4),
              "inliers_rel_diff_median_on_valid": round(float(np.median(rel_in)), 4) if both.any() else None,
              "inliers_rel_diff_max_on_valid": round(float(rel_in.max()), 4) if both.any() else None,
              "seconds": round(time.time() - t0, 1)}
    print(json.dumps(report, indent=1))
    if a.out:
        out = {k: g[k] for k in g}
        out.update({"fp32_matches": ref_n, "fp32_inliers": ref_in, "fp32_is_valid": ref_valid, "fp32_stop": ref_stop,
                    "report": np.array(json.dumps(report))})
        np.savez_compressed(a.out, **out)


if __name__ == "__main__":
    main()
