"""World-size-2 gloo test of the frame-parallel path (CPU): sharding, the descriptor
all-gather and the row-sharded retrieval must reproduce the single-process result.
The per-rank retrieval compute here is the oracle (no GPU in this test); on the GPU
box the same plumbing drives the HIP kernels (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mlgate import distributed as mdist


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, d, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import _lib, retrieval as oret
    rng = np.random.default_rng(0)
    X = rng.standard_normal((40, d)).astype(np.float32)[rng.integers(0, 40, n)]
    X = X + 0.7 * rng.standard_normal((n, d)).astype(np.float32)
    t = np.arange(n) * 0.765
    fl = np.repeat(np.array([5, 1, 4, 2], np.int64), [n // 4, n // 4, n // 4, n - 3 * (n // 4)])
    hf = np.ones(n, np.uint8)
    lo, hi = mdist.shard(n, world, rank)
    local = torch.from_numpy(X[lo:hi])  # this rank's "extracted" descriptors
    gather = mdist.RowGather(n, d, world, "cpu")
    full = gather(local).numpy()
    assert np.array_equal(full, X)
    S = oret.pairwise_similarities(full)[lo:hi]
    idx, sim, valid, count = _lib.knn_rows(S, lo, t, fl, hf, 10.0, 0.5, 10, True)
    sel = np.arange(10)[None, :] < count[:, None]
    part = (np.repeat(np.arange(lo, hi), count), idx[sel].astype(np.int64), sim[sel], valid[sel])
    parts = mdist.gather_objects_to_rank0(part, world, rank)
    if rank == 0:
        merged = mdist.merge_matches(parts)
        ref = oret.find_loop_closures(X, t, fl, hf, 10.0, 0.5, 10, True)
        ok = all(np.array_equal(a, b) for a, b in zip(merged, ref)) and len(merged[0]) > 0
        with open(out_path, "w") as f:
            f.write("ok" if ok else "mismatch")
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [301, 1000])
def test_row_sharded_gate_equals_single_process(tmp_path, n):
    out = str(tmp_path / "result.txt")
    mp.spawn(_worker, args=(2, _free_port(), n, 64, out), nprocs=2, join=True)
    assert open(out).read() == "ok"


def test_shards_cover_exactly():
    for n in (1, 7, 5000, 19163):
        for w in (1, 2, 4, 8):
            rs = [mdist.shard(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert sum(mdist.shard_sizes(n, w)) == n


def _pairs_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(rank)
    n = [7, 0, 23][rank]  # deliberately uneven (and one empty) per-rank pair lists
    pa = torch.from_numpy((1000 * rank + np.arange(n)).astype(np.int32))
    pb = torch.from_numpy(rng.integers(0, 100, n).astype(np.int32))
    sa, sb = mdist.balanced_pairs(pa, pb, world, rank)
    got = mdist.gather_objects_to_rank0((sa.numpy(), sb.numpy()), world, rank)
    full = mdist.gather_objects_to_rank0((pa.numpy(), pb.numpy()), world, rank)
    if rank == 0:
        ga = np.concatenate([g[0] for g in got])
        gb = np.concatenate([g[1] for g in got])
        fa = np.concatenate([f[0] for f in full])
        fb = np.concatenate([f[1] for f in full])
        sizes = [len(g[0]) for g in got]
        ok = np.array_equal(ga, fa) and np.array_equal(gb, fb) and max(sizes) - min(sizes) <= 1
        with open(out_path, "w") as f:
            f.write("ok" if ok else f"mismatch {sizes}")
    dist.destroy_process_group()


def test_balanced_pairs_partition_the_global_list(tmp_path):
    """Verification pairs re-split across ranks: union == the rank-ordered global list,
    slice sizes within one of each other (bench.py's multi-GPU verification stage)."""
    out = str(tmp_path / "pairs.txt")
    mp.spawn(_pairs_worker, args=(3, _free_port(), out), nprocs=3, join=True)
    assert open(out).read() == "ok"


def _pairs_rev_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(10 + rank)
    n = [40, 0, 57][rank]
    pa = rng.integers(0, 30, n).astype(np.int32)
    pb = rng.integers(0, 30, n).astype(np.int32)
    if rank == 2:  # reverses of rank 0's pairs, found by another rank's queries
        r0 = np.random.default_rng(10)
        a0, b0 = r0.integers(0, 30, 40).astype(np.int32), r0.integers(0, 30, 40).astype(np.int32)
        pa[:20], pb[:20] = b0[:20], a0[:20]
    sa, sb = mdist.balanced_pairs(torch.from_numpy(pa), torch.from_numpy(pb), world, rank, group_reverse=True)
    got = mdist.gather_objects_to_rank0((sa.numpy(), sb.numpy()), world, rank)
    full = mdist.gather_objects_to_rank0((pa, pb), world, rank)
    if rank == 0:
        allp = sorted(zip(np.concatenate([f[0] for f in full]).tolist(), np.concatenate([f[1] for f in full]).tolist()))
        gotp = sorted(p for g in got for p in zip(g[0].tolist(), g[1].tolist()))
        owner = {}
        clash = False
        for r, g in enumerate(got):
            for a, b in zip(g[0].tolist(), g[1].tolist()):
                k = (min(a, b), max(a, b))
                clash |= owner.setdefault(k, r) != r
        per_rank = [len({(min(a, b), max(a, b)) for a, b in zip(g[0].tolist(), g[1].tolist())}) for g in got]
        ok = gotp == allp and not clash and max(per_rank) - min(per_rank) <= 1
        with open(out_path, "w") as f:
            f.write("ok" if ok else f"mismatch clash={clash} {per_rank}")
    dist.destroy_process_group()


def test_balanced_pairs_group_reverse(tmp_path):
    """group_reverse: the union is still the global pair multiset, (a, b) and (b, a) land
    on one rank (matched once there), unordered pairs split within one of each other."""
    out = str(tmp_path / "pairs_rev.txt")
    mp.spawn(_pairs_rev_worker, args=(3, _free_port(), out), nprocs=3, join=True)
    assert open(out).read() == "ok"


def _fx_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 53
    full_kp = torch.arange(n * 6, dtype=torch.float32).view(n, 6) * 0.5
    full_ds = torch.randn(n, 16, generator=torch.Generator().manual_seed(7))
    full_cnt = torch.arange(n, dtype=torch.int32).view(n, 1) * 3
    lo, hi = mdist.shard(n, world, rank)
    rng = np.random.default_rng(100 + rank)
    need = np.unique(rng.integers(0, n, [17, 0, 40][rank]))  # uneven, one rank needs nothing
    fx = mdist.FeatureExchange(n, world, rank)
    kp, ds, cnt = fx(need, [full_kp[lo:hi], full_ds[lo:hi], full_cnt[lo:hi]])
    idx = torch.from_numpy(need.astype(np.int64))
    ok = (torch.equal(kp, full_kp[idx]) and torch.equal(ds, full_ds[idx]) and torch.equal(cnt, full_cnt[idx])
          and fx.last_bytes == len(need) * (6 * 4 + 16 * 4 + 4))
    res = mdist.gather_objects_to_rank0(bool(ok), world, rank)
    if rank == 0:
        with open(out_path, "w") as f:
            f.write("ok" if all(res) else f"mismatch {res}")
    dist.destroy_process_group()


def test_feature_exchange_delivers_exactly_the_needed_rows(tmp_path):
    """FeatureExchange (the sharded gate's SuperPoint feature step): each rank receives the
    rows of exactly the keyframes it asked for, in ascending global order, from whichever
    ranks own them -- uneven needs, an empty need list, several dtypes."""
    out = str(tmp_path / "fx.txt")
    mp.spawn(_fx_worker, args=(3, _free_port(), out), nprocs=3, join=True)
    assert open(out).read() == "ok"


def _w8_worker(rank, world, port, out_path):
    """Everything the sharded gate exchanges, at the node's size (W = 8): the descriptor
    all-gather at N = 5000 (625 rows per rank: the equal-shard all_gather_into_tensor RCCL
    gets) and at N = 5003 (uneven: padded all_gather + compaction), balanced_pairs with
    group_reverse over 8 slices (reverse pairs found by other ranks' queries), and
    FeatureExchange with 8 senders and receivers (uneven and empty need lists)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    errs = []
    for n in (5000, 5003):
        X = torch.from_numpy(np.random.default_rng(n).standard_normal((n, 48)).astype(np.float32))
        lo, hi = mdist.shard(n, world, rank)
        g = mdist.RowGather(n, 48, world, "cpu")
        if not torch.equal(g(X[lo:hi].clone()), X):
            errs.append(f"rowgather {n}")
        if n == 5000 and not (len(set(g.sizes)) == 1 and g.sizes[0] == 625):
            errs.append("shards")
    # pairs: each rank's queries are its own keyframes; ~1/3 of the pairs also appear
    # reversed on the rank owning the match (the kNN returns most revisits both ways)
    n = 400
    lo, hi = mdist.shard(n, world, rank)
    allq = []
    for r in range(world):
        rr = np.random.default_rng(50 + r)
        l_, h_ = mdist.shard(n, world, r)
        q = rr.integers(l_, h_, 60)
        m = rr.integers(0, n, 60)
        allq.append((q, m))
    extra = [(m[:20], q[:20]) for q, m in allq]  # the reverses
    qa = np.concatenate([allq[rank][0]] + [e[0][(e[0] >= lo) & (e[0] < hi)] for e in extra]).astype(np.int32)
    qb = np.concatenate([allq[rank][1]] + [e[1][(e[0] >= lo) & (e[0] < hi)] for e in extra]).astype(np.int32)
    if rank == 3:
        qa, qb = qa[:0], qb[:0]  # one rank found nothing
    sa, sb = mdist.balanced_pairs(torch.from_numpy(qa), torch.from_numpy(qb), world, rank, group_reverse=True)
    got = mdist.gather_objects_to_rank0((sa.numpy(), sb.numpy()), world, rank)
    full = mdist.gather_objects_to_rank0((qa, qb), world, rank)
    # features: 8 senders, needs drawn from this rank's pair slice (+ one empty rank)
    kp = torch.arange(n * 4, dtype=torch.float32).view(n, 4) * 0.25
    ds = torch.randn(n, 8, generator=torch.Generator().manual_seed(3))
    need = np.unique(np.concatenate([sa.numpy(), sb.numpy()]).astype(np.int64)) if rank != 5 else np.zeros(0, np.int64)
    fx = mdist.FeatureExchange(n, world, rank)
    rk, rd = fx(need, [kp[lo:hi], ds[lo:hi]])
    idx = torch.from_numpy(need)
    if not (torch.equal(rk, kp[idx]) and torch.equal(rd, ds[idx])):
        errs.append(f"fx rank {rank}")
    res = mdist.gather_objects_to_rank0(errs, world, rank)
    if rank == 0:
        allp = sorted(zip(np.concatenate([f[0] for f in full]).tolist(), np.concatenate([f[1] for f in full]).tolist()))
        gotp = sorted(p for g_ in got for p in zip(g_[0].tolist(), g_[1].tolist()))
        owner, clash = {}, False
        for r, g_ in enumerate(got):
            for a, b in zip(g_[0].tolist(), g_[1].tolist()):
                clash |= owner.setdefault((min(a, b), max(a, b)), r) != r
        per_rank = [len({(min(a, b), max(a, b)) for a, b in zip(g_[0].tolist(), g_[1].tolist())}) for g_ in got]
        errs_all = [e for r in res for e in r]
        if gotp != allp:
            errs_all.append("pairs union")
        if clash or max(per_rank) - min(per_rank) > 1:
            errs_all.append(f"pairs split clash={clash} {per_rank}")
        with open(out_path, "w") as f:
            f.write("ok" if not errs_all else "; ".join(errs_all))
    dist.destroy_process_group()


def test_world8_exchanges(tmp_path):
    """the sharded gate's three exchanges at W = 8 (gloo on the CPU;
    RCCL's device transport itself needs a node and stays unmeasured here)."""
    out = str(tmp_path / "w8.txt")
    mp.spawn(_w8_worker, args=(8, _free_port(), out), nprocs=8, join=True)
    assert open(out).read() == "ok"
