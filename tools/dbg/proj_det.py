"""Diagnostic: run-to-run determinism of mlg_op_lg_proj (self and cross) over many runs."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "multi-level-indoor-slam_amd")]
from mlgate import _native  # noqa: E402
from mlgate.lightglue import pack_kstep  # noqa: E402

dev = torch.device("cuda:0")
L = _native.lib()
P = lambda t: __import__("ctypes").c_void_p(t.data_ptr())  # noqa: E731
Npad, H, runs = 65536, 4, int(os.environ.get("RUNS", "20"))
g = torch.Generator().manual_seed(11)
xc = torch.zeros(Npad, 512, dtype=torch.bfloat16)
xc[:, :256] = torch.randn(Npad, 256, generator=g).to(torch.bfloat16)
for self_block in (1, 0):
    N = 768 if self_block else 512
    W = torch.from_numpy(pack_kstep((torch.randn(N, 256, generator=g) / 16).numpy())).to(torch.bfloat16)
    b = torch.randn(N, generator=g) * 0.1
    ang = torch.rand(Npad, 32, generator=g) * 6.3
    live = (torch.rand(Npad, generator=g) > 0.1).to(torch.uint8)
    d = {k: v.to(dev) for k, v in dict(xc=xc, W=W, b=b, ec=torch.cos(ang), es=torch.sin(ang), live=live).items()}
    ref, bad = None, {"Q": 0, "K": 0, "V": 0}
    for r in range(runs):
        Q = torch.zeros(H, Npad, 64, dtype=torch.bfloat16, device=dev)
        K = torch.zeros_like(Q)
        Vt = torch.zeros(H, Npad // 64, 64, 64, dtype=torch.bfloat16, device=dev)
        _native.check(L.mlg_op_lg_proj(self_block, P(d["xc"]), 512, P(d["W"]), P(d["b"]), P(d["ec"]), P(d["es"]),
                                       P(d["live"]), P(Q), P(K), P(Vt), Npad, _native.stream_of(dev)), "proj")
        torch.cuda.synchronize()
        out = {"Q": Q, "K": K, "V": Vt}
        if ref is None:
            ref = {k: v.clone() for k, v in out.items()}
            continue
        for k in out:
            if not torch.equal(out[k], ref[k]):
                bad[k] += 1
                if bad[k] == 1:
                    diff = (out[k] != ref[k]).nonzero()
                    print("self" if self_block else "cross", k, "first diff rows", diff[:4].tolist(), len(diff))
    print("self" if self_block else "cross", "mismatching runs of", runs - 1, bad, flush=True)
