"""Are the bench's per-rank inputs and descriptors those of the single-rank run, bit for bit?

    python tools/shard_diag.py [--n 5000]

(A) the whole sequence's frames and split-ViT descriptors in one pass (bench.py's batch 246);
(B) each rank's shard at W = 2 and 4 rendered and described on its own, one after another;
(C) the W = 4 shards described by four processes at once on the one GPU (co-scheduled
    kernels, as the MLGATE_BENCH_REHEARSE bench runs them).
Prints, per case, how many shard rows differ from (A) and by how much."""
import argparse
import json
import os
import sys
import tempfile

import numpy as np
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-level-indoor-slam_amd")]


def _describe(lo, hi, n, places, batch):
    import bench
    from mlgate import synthetic
    from mlgate.vit import VitB14
    from mlgate.weights import synthetic_state_dict
    seq, _ = bench.sequence(n, places)
    fr = synthetic.frames_device(seq, np.arange(lo, hi), torch.device("cuda", 0))
    eng = VitB14(synthetic_state_dict(0), device="cuda", max_batch=batch, precise=True)
    d = eng.forward(fr)
    torch.cuda.synchronize()
    return fr, d


def _worker(rank, world, n, places, batch, out):
    torch.cuda.set_device(0)
    from mlgate import distributed as mdist
    lo, hi = mdist.shard(n, world, rank)
    _, d = _describe(lo, hi, n, places, batch)
    np.save(os.path.join(out, f"d{rank}.npy"), d.cpu().numpy())


def _sequential_equal(fr, n, places):
    """the first frames against one seeded stream drawn frame after frame (the generator
    as frames_device used it before the per-frame offsets): the single-rank workload kept"""
    import bench
    from mlgate import synthetic
    seq, _ = bench.sequence(n, places)
    dev = fr.device
    g = torch.Generator(device=dev).manual_seed(seq.seed)
    for i in range(fr.shape[0]):
        base = torch.from_numpy(synthetic._base(int(seq.place_of[i]), synthetic.H, synthetic.W)).to(dev)
        sx, sy = (int(v) for v in seq.shift[i])
        f = torch.roll(base, shifts=(sy, sx), dims=(0, 1)).to(torch.int16)
        f = (f + torch.randint(0, 30, f.shape, generator=g, device=dev, dtype=torch.int16)).clamp_(0, 255)
        if not torch.equal(f.to(torch.uint8), fr[i]):
            return False
    return True


def _cmp(ref, got):
    diff = (ref != got).any(dim=1)
    return {"rows": int(ref.shape[0]), "rows_differing": int(diff.sum()),
            "max_abs": float((ref - got).abs().max()) if diff.any() else 0.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=5000)
    ap.add_argument("--places", type=int, default=600)
    ap.add_argument("--batch", type=int, default=246)
    a = ap.parse_args()
    from mlgate import distributed as mdist
    frA, dA = _describe(0, a.n, a.n, a.places, a.batch)
    res = {"A_first64_equal_sequential_stream": _sequential_equal(frA[:64], a.n, a.places)}
    for W in (2, 4):
        for r in range(W):
            lo, hi = mdist.shard(a.n, W, r)
            fr, d = _describe(lo, hi, a.n, a.places, a.batch)
            res[f"B_w{W}_r{r}"] = dict(frames_equal=bool(torch.equal(fr, frA[lo:hi])), **_cmp(dA[lo:hi], d))
            del fr, d
    torch.cuda.empty_cache()
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(4, a.n, a.places, a.batch, td), nprocs=4, join=True)
        for r in range(4):
            lo, hi = mdist.shard(a.n, 4, r)
            d = torch.from_numpy(np.load(os.path.join(td, f"d{r}.npy"))).to(dA.device)
            res[f"C_w4_r{r}_concurrent"] = _cmp(dA[lo:hi], d)
    for k, v in res.items():
        print(json.dumps({"case": k, **v} if isinstance(v, dict) else {"case": k, "value": v}), flush=True)


if __name__ == "__main__":
    main()
