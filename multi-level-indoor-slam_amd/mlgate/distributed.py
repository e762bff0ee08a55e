"""Frame-parallel multi-GPU gate: one process per GPU, torch.distributed over RCCL
("nccl" backend on ROCm) or gloo (CPU tests).

The only exchange step of the path is the descriptor all-gather before retrieval
(SURVEY.md §8e): each rank extracts descriptors for its own contiguous shard of
keyframes, all ranks all-gather the [N/W, D] float32 rows into the full database, and
each rank ranks its own query rows against it.  Rows are independent, so the union of
the per-rank outputs, in rank order, is exactly the single-GPU output.
"""
import numpy as np
import torch
import torch.distributed as dist


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
        self.send[:local.shape[0]].copy_(local)
        dist.all_gather(self.bufs, self.send, group=self.group)
        torch.cat([b[:s] for b, s in zip(self.bufs, self.sizes)], out=self.out)
        return self.out


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
