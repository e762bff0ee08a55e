"""Frame-parallel multi-GPU gate: one process per GPU, torch.distributed over RCCL
("nccl" backend on ROCm) or gloo (CPU tests).

Exchange steps of the path: the descriptor all-gather before retrieval
-- each rank extracts descriptors for its own contiguous shard of keyframes, all ranks
all-gather the [N/W, D] float32 rows into the full database, and each rank ranks its own
query rows against it (rows are independent, so the union of the per-rank outputs, in
rank order, is exactly the single-GPU output); an 8-B-per-pair all-gather that
re-balances the verification pairs (balanced_pairs); and a need-driven exchange of the
SuperPoint features of the keyframes each rank's pairs touch (FeatureExchange).
"""
import numpy as np
import torch
import torch.distributed as dist


def _staged(t, group=None):
    """gloo cannot reduce or gather HIP tensors: collectives on device tensors go through
    host copies when the process group is gloo (the CPU / one-GPU multi-rank tests); RCCL
    ("nccl") takes the device tensors directly."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_gather_into(bufs, send, group=None):
    if _staged(send, group):
        hb = [torch.empty(b.shape, dtype=b.dtype) for b in bufs]
        dist.all_gather(hb, send.cpu(), group=group)
        for b, h in zip(bufs, hb):
            b.copy_(h)
    else:
        dist.all_gather(bufs, send, group=group)


def all_reduce_(t, group=None):
    if _staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)
    return t


def shard(n, world, rank):
    """Contiguous keyframe range [lo, hi) owned by `rank`."""
    return rank * n // world, (rank + 1) * n // world


def shard_sizes(n, world):
    return [shard(n, world, r)[1] - shard(n, world, r)[0] for r in range(world)]


class RowGather:
    """All-gather of unevenly sharded rows into one [N, D] tensor (buffers reused)."""

    def __init__(self, n, d, world, device, dtype=torch.float32, group=None):
        self.sizes = shard_sizes(n, world)
        self.pad = max(self.sizes)
        self.group = group
        self.bufs = [torch.empty(self.pad, d, dtype=dtype, device=device) for _ in range(world)]
        self.send = torch.empty(self.pad, d, dtype=dtype, device=device)
        self.out = torch.empty(n, d, dtype=dtype, device=device)

    def __call__(self, local):
        if len(self.sizes) == 1:
            self.out.copy_(local)
            return self.out
        if len(set(self.sizes)) == 1 and not _staged(local, self.group):
            # equal shards (N % W == 0, e.g. 5000 over 1 / 2 / 4 / 8 ranks): one all-gather
            # straight into the [N, D] database, no staging copy -- RCCL on device tensors,
            # and the very same call on host tensors under gloo (the world-size-2 CPU test
            # with N = 1000 runs this branch, tests/test_distributed.py)
            dist.all_gather_into_tensor(self.out, local.contiguous(), group=self.group)
            return self.out
        self.send[:local.shape[0]].copy_(local)
        all_gather_into(self.bufs, self.send, group=self.group)
        torch.cat([b[:s] for b, s in zip(self.bufs, self.sizes)], out=self.out)
        return self.out


def balanced_pairs(pa, pb, world, rank, group=None, group_reverse=False):
    """Pair-level load balance for the verification stage.  Each rank holds the
    gate-accepted (query, match) pairs of its own query rows (int32 tensors, row-major
    order); their number varies with the floor layout and the revisit pattern, so
    verifying them where they were found leaves ranks idle.  All ranks all-gather the
    lists (8 B per pair) and take the rank-th contiguous slice of the global,
    rank-ordered list: the union of the slices is exactly the global list and slice
    sizes differ by at most one.  FeatureExchange then delivers each rank the features
    (or frames) of exactly the keyframes its slice touches.
    With ``group_reverse`` the slices are cut over the UNORDERED pairs instead: (a, b) and
    (b, a) land on the same rank, which matches them once (LightGlue is symmetric in its
    two images; mlg_lg_orient_matches); the unordered pairs are split evenly, in
    ascending (min, max) order."""
    if world == 1:
        return pa, pb
    dev = pa.device
    n = torch.tensor([pa.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    all_gather_into(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    pad = max(max(sizes), 1)
    send = torch.zeros(2, pad, dtype=torch.int32, device=dev)
    send[0, :pa.numel()] = pa
    send[1, :pb.numel()] = pb
    bufs = [torch.empty_like(send) for _ in range(world)]
    all_gather_into(bufs, send, group=group)
    allp = torch.cat([b[:, :s] for b, s in zip(bufs, sizes)], dim=1)
    if group_reverse:
        lo_ = torch.minimum(allp[0], allp[1]).long()
        hi_ = torch.maximum(allp[0], allp[1]).long()
        span = int(hi_.max().item()) + 1 if hi_.numel() else 1
        ukey, inv = torch.unique(lo_ * span + hi_, sorted=True, return_inverse=True)
        nu = ukey.numel()
        ulo, uhi = rank * nu // world, (rank + 1) * nu // world
        sel = torch.nonzero((inv >= ulo) & (inv < uhi), as_tuple=True)[0]
        return allp[0, sel].contiguous(), allp[1, sel].contiguous()
    total = allp.shape[1]
    lo, hi = rank * total // world, (rank + 1) * total // world
    return allp[0, lo:hi].contiguous(), allp[1, lo:hi].contiguous()


class FeatureExchange:
    """The SuperPoint feature exchange of the sharded gate: every rank receives exactly the
    keyframes its verification slice needs (not the whole [N, 2048, 256] table).  Rank r
    owns keyframes shard(n, W, r); given the sorted global indices `need` this rank
    verifies against, it all-gathers the (tiny) need lists, sends every requester the
    rows of its own shard that requester needs, and receives its own needs, in ascending
    global order, through one all_to_all per feature tensor (RCCL over xGMI; gloo through
    host copies).  Row k of each returned tensor is keyframe need[k]."""

    def __init__(self, n, world, rank, group=None):
        self.n, self.world, self.rank, self.group = n, world, rank, group
        self.bounds = [shard(n, world, r) for r in range(world)]

    def _gather_needs(self, need, dev):
        k = torch.tensor([len(need)], dtype=torch.int64, device=dev)
        sizes = [torch.zeros_like(k) for _ in range(self.world)]
        all_gather_into(sizes, k, group=self.group)
        sizes = [int(x.item()) for x in sizes]
        pad = max(max(sizes), 1)
        send = torch.full((pad,), -1, dtype=torch.int64, device=dev)
        send[:len(need)] = torch.from_numpy(np.asarray(need, np.int64)).to(dev)
        bufs = [torch.empty_like(send) for _ in range(self.world)]
        all_gather_into(bufs, send, group=self.group)
        return [b[:s].cpu().numpy() for b, s in zip(bufs, sizes)]

    def __call__(self, need, tensors):
        """need: sorted unique int64 global keyframe indices; tensors: local per-keyframe
        tensors [n_local, ...] (this rank's shard, in order).  Returns tensors [len(need), ...]."""
        need = np.asarray(need, np.int64)
        dev = tensors[0].device
        lo, hi = self.bounds[self.rank]
        needs = self._gather_needs(need, dev)
        # rows of my shard each requester wants, requester order; and my receive counts
        send_rows = [nr[(nr >= lo) & (nr < hi)] - lo for nr in needs]
        in_splits = [len(x) for x in send_rows]
        out_splits = [int(((need >= a) & (need < b)).sum()) for a, b in self.bounds]
        idx = torch.from_numpy(np.concatenate(send_rows).astype(np.int64)).to(dev)
        out = []
        for t in tensors:
            send = t.index_select(0, idx).contiguous()
            recv = torch.empty((len(need),) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
            if _staged(send, self.group):
                h = torch.empty(recv.shape, dtype=recv.dtype)
                dist.all_to_all_single(h, send.cpu(), out_splits, in_splits, group=self.group)
                recv.copy_(h)
            else:
                dist.all_to_all_single(recv, send, out_splits, in_splits, group=self.group)
            out.append(recv)
        self.last_bytes = sum(int(o.numel()) * o.element_size() for o in out)
        return out


def gather_objects_to_rank0(obj, world, rank, group=None):
    """Python objects (e.g. per-rank match arrays) collected on rank 0, in rank order."""
    if world == 1:
        return [obj]
    out = [None] * world if rank == 0 else None
    dist.gather_object(obj, out, dst=0, group=group)
    return out


def merge_matches(parts):
    """Concatenate per-rank flat (q, m, sim, valid) arrays in rank order."""
    return tuple(np.concatenate([p[i] for p in parts]) for i in range(4))
