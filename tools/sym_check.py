"""How symmetric is the verified pair set, and is LightGlue(b, a) the swap of
LightGlue(a, b) on this implementation?  (GPU box tool.)

    python tools/sym_check.py [--keyframes 5000] [--sample 1024]

Runs bench.py's DeviceGate once, counts pairs whose reverse is also verified, then
matches a sample of such pairs in both orders and compares the match sets (as
unordered index pairs), the scores and the stop layers, and the RANSAC decisions of
the reference's rule on each order."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from mlgate import geometry, synthetic  # noqa: E402
from mlgate.pipeline import DeviceGate  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keyframes", type=int, default=5000)
    ap.add_argument("--sample", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    seq, labels = bench.sequence(a.keyframes, 600)
    frames = synthetic.frames_device(seq, np.arange(a.keyframes), dev)
    gate = DeviceGate(frames, seq.t, labels, 1, 0, dev, k=20, verify=True, K=bench.ISEC_K, vit_batch=123, sp_batch=64,
                      lg_chunk=1024, vit_state_dict=synthetic_state_dict(0))
    counts = gate.step()
    pa, pb = gate.last_pairs
    fwd = set(zip(pa.tolist(), pb.tolist()))
    sym = [(x, y) for x, y in fwd if (y, x) in fwd]
    uniq = {(min(x, y), max(x, y)) for x, y in fwd}
    res = {"pairs": len(fwd), "pairs_with_reverse": len(sym), "unordered_unique": len(uniq), "counts": counts}
    smp = sorted({(min(x, y), max(x, y)) for x, y in sym})[:a.sample]
    A = np.array([x for x, _ in smp], np.int32)
    B = np.array([y for _, y in smp], np.int32)
    kp_all = gate.kp_loc.view(gate.N, gate.kp, 2)
    ds_all = gate.ds_loc.view(gate.N, gate.kp, 256)
    cnt = gate.cnt_loc.view(-1).cpu().numpy()
    m1, s1, n1, st1 = gate.lg.match_device(kp_all, ds_all, cnt, A, B)
    m2, s2, n2, st2 = gate.lg.match_device(kp_all, ds_all, cnt, B, A)
    m1, s1, n1, m2, s2, n2 = (t.cpu().numpy() for t in (m1, s1, n1, m2, s2, n2))
    same_set = same_order_after_sort = same_stop = 0
    max_sdiff = 0.0
    for p in range(len(smp)):
        e1 = {(int(u), int(v)): float(sc) for (u, v), sc in zip(m1[p, :n1[p]], s1[p, :n1[p]])}
        e2 = {(int(v), int(u)): float(sc) for (u, v), sc in zip(m2[p, :n2[p]], s2[p, :n2[p]])}
        if set(e1) == set(e2):
            same_set += 1
            max_sdiff = max([max_sdiff] + [abs(e1[k] - e2[k]) for k in e1])
            sw = sorted(((v, u) for u, v in e1), key=lambda t: t[0])
            same_order_after_sort += sw == [(int(u), int(v)) for u, v in m2[p, :n2[p]]]
        same_stop += int(st1[p] == st2[p])
    res.update({"sample": len(smp), "same_match_set": same_set, "same_order_after_swap_sort": same_order_after_sort,
                "same_stop_layer": same_stop, "max_score_diff_on_same_sets": max_sdiff})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
