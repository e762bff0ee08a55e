"""RCCL ("nccl" on ROCm) executing the sharded gate's device collectives on the GPU.

No multi-GPU node is available to this build, and RCCL will not put two ranks on one
device, so the collectives run with ONE rank: RCCL's own device path (communicator set-up,
the kernels, the self-send) on the very calls the sharded gate makes -- the equal-shard
descriptor `all_gather_into_tensor` of mlgate.distributed.RowGather and the
`all_to_all_single` of FeatureExchange on device tensors (no host staging: the staged
branch is gloo's) -- with results checked.  The multi-rank transport over xGMI stays
unmeasured; the multi-rank logic is covered by the gloo tests at W = 2, 3
and 8 (tests/test_distributed.py) and by DeviceGate at W = 2 and 4 on one GPU
(tests/test_distributed_gpu.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from mlgate import distributed as mdist
    errs = []
    try:
        assert dist.get_backend() == "nccl"
        # RowGather's equal-shard path: one all_gather_into_tensor straight into [N, D]
        x = torch.randn(625, 768, device=dev)
        out = torch.empty(625, 768, device=dev)
        assert not mdist._staged(x)
        dist.all_gather_into_tensor(out, x)
        if not torch.equal(out, x):
            errs.append("all_gather_into_tensor")
        # FeatureExchange (no world-1 shortcut): need-list all-gather + all_to_all_single of
        # f32 keypoints / descriptors and int32 counts on the device
        n = 300
        kp = torch.randn(n, 4096, device=dev)
        ds = torch.randn(n, 2048, device=dev)
        cnt = torch.arange(n, dtype=torch.int32, device=dev).view(n, 1)
        need = torch.randperm(n)[:117].sort().values.numpy()
        fx = mdist.FeatureExchange(n, 1, 0)
        rk, rd, rc = fx(need, [kp, ds, cnt])
        idx = torch.from_numpy(need).to(dev)
        if not (torch.equal(rk, kp[idx]) and torch.equal(rd, ds[idx]) and torch.equal(rc, cnt[idx])):
            errs.append("FeatureExchange")
        # the verdict totals' all-reduce
        t = torch.tensor([3, 4], dtype=torch.int64, device=dev)
        mdist.all_reduce_(t)
        if t.tolist() != [3, 4]:
            errs.append("all_reduce")
        torch.cuda.synchronize()
    except Exception as e:  # reported through the file: mp.spawn's own error is opaque
        errs.append(repr(e))
    with open(out_path, "w") as f:
        f.write("ok" if not errs else "; ".join(errs))
    dist.destroy_process_group()


def test_rccl_device_collectives_one_rank(tmp_path):
    out = str(tmp_path / "rccl.txt")
    mp.spawn(_worker, args=(_free_port(), out), nprocs=1, join=True)
    assert open(out).read() == "ok"
