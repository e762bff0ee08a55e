"""Host-side pieces of bench.py and tools/bench_parity.py (no GPU): the LoFTR FLOP
accounting, the collectives helper of the multi-rank flow under gloo (the one-GPU
rehearsal's backend), and the GPU-vs-C-twin model comparison."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import bench  # noqa: E402


def test_loftr_flops_count_layer0_at_its_sides():
    """8 coarse layers on both sides when layer 0 runs per pair side (the reference's
    count); with layer 0 once per distinct frame the count drops by exactly that layer's
    share; the L^2 similarity and the fine stage are unchanged."""
    L, m = 4800, 120.0
    lay = bench._lf_layer_flops(256)
    ref = 8 * 2 * L * lay + 2 * L * L * 256 + m * 2 * 2 * 25 * bench._lf_layer_flops(128)
    assert bench.loftr_flops_per_pair(L, m) == ref
    assert bench.loftr_flops_per_pair(L, m, 1.25) == ref - 0.75 * L * lay
    assert bench._lf_layer_flops(256) == 2 * (4 * 256 * 256 + 2 * 256 * 512 + 2 * 256 * 256 + 2 * 8 * 32 * 32)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reduce_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([1.5 + rank, 10.0 * rank], dtype=torch.float64)
    c = torch.tensor([3, rank], dtype=torch.int64)
    bench._all_reduce(t, dist.ReduceOp.MAX)
    bench._all_reduce(c)
    if rank == 0:
        np.save(out, np.concatenate([t.numpy(), c.numpy().astype(np.float64)]))
    dist.destroy_process_group()


def test_all_reduce_helper_under_gloo(tmp_path):
    """bench.py's in-place all-reduce (host-staged under gloo, as the one-GPU rehearsal runs
    it): MAX of the step times, SUM of the counts, at world size 3."""
    out = str(tmp_path / "r.npy")
    mp.spawn(_reduce_worker, args=(3, _free_port(), out), nprocs=3, join=True)
    assert np.load(out).tolist() == [3.5, 20.0, 9.0, 3.0]


def test_same_model_compares_bits():
    import bench_parity as bp
    M = np.arange(9, dtype=np.float64).reshape(3, 3) / 7.0
    assert bp._same_model(M, M.copy())
    assert bp._same_model(None, None)
    assert not bp._same_model(M, None) and not bp._same_model(None, M)
    N = M.copy()
    N[1, 1] = np.nextafter(N[1, 1], 2.0)  # one ulp
    assert not bp._same_model(M, N)
    Z = np.zeros((3, 3))
    assert not bp._same_model(Z, -Z)  # +0 and -0 differ in their bits
