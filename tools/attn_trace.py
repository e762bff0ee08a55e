"""Phase timeline of the LightGlue attention tile (attention.hip) from a -DMLG_ATT_TRACE=1
build (GPU box tool, through tools/ab_run.py --lib-dir <trace build>): one ragged launch
(n segments of L tokens, H heads, self tasks), then per workgroup the s_memtime stamps at
entry, after the prologue (Q fragments, the first K / V stages in LDS), after the stage
loop, and at the end (O normalised, staged, stored), with the CU it ran on.  Prints the
median cycles of each phase, the share of a workgroup's time outside the stage loop, and
the gap between one workgroup's end and the next one's start on the same CU.

    python tools/ab_run.py --lib-dir ab_attt tools/attn_trace.py [--n 200 --L 2048 --H 4]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
from mlgate import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--L", type=int, default=2048)
    ap.add_argument("--H", type=int, default=4)
    a = ap.parse_args()
    lib = _native.lib()
    dev = torch.device("cuda:0")
    n, L, H = a.n, a.L, a.H
    Lp = (L + 63) // 64 * 64
    g = torch.Generator(device=dev).manual_seed(0)
    Q = (torch.randn(H, n, Lp, 64, generator=g, device=dev) * 1.5).to(torch.bfloat16)
    K = (torch.randn(H, n, Lp, 64, generator=g, device=dev) * 1.5).to(torch.bfloat16)
    V = torch.randn(H, n, Lp, 64, generator=g, device=dev) * 1.5
    V[:, :, L:] = 0
    Vt = V.to(torch.bfloat16).reshape(H, n * Lp // 64, 64, 64).transpose(-1, -2).contiguous()
    tasks = torch.tensor([[i * Lp, L, i * Lp, L] for i in range(n)], dtype=torch.int32, device=dev)
    oo = torch.tensor([i * Lp for i in range(n)], dtype=torch.int32, device=dev)
    O = torch.zeros((n * Lp, H * 64), dtype=torch.bfloat16, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    vp = ctypes.c_void_p
    for _ in range(3):
        rc = lib.mlg_op_attention_varlen(vp(Q.data_ptr()), vp(K.data_ptr()), vp(Vt.data_ptr()), vp(O.data_ptr()),
                                         H * 64, n * Lp, H, vp(tasks.data_ptr()), vp(oo.data_ptr()), n, L, st)
        assert rc == 0
    torch.cuda.synchronize()
    buf = np.zeros((1 << 16, 8), np.uint64)
    if lib.mlg_dbg_att_trace(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) != 0:
        raise SystemExit("not a -DMLG_ATT_TRACE=1 build")
    tr = buf[buf[:, 7] == 1].astype(np.int64)
    t = tr[:, :4]
    d = np.diff(t, axis=1)
    total = t[:, 3] - t[:, 0]
    hw, xcc = tr[:, 4], tr[:, 5]
    cu = (xcc & 15) * 4096 + ((hw >> 13) & 7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 15)
    gaps = []
    for k in np.unique(cu):
        idx = np.flatnonzero(cu == k)
        idx = idx[np.argsort(t[idx, 0])]
        gaps.extend((t[idx[1:], 0] - t[idx[:-1], 3]).tolist())
    res = {"n": n, "L": L, "H": H, "workgroups": int(len(t)),
           "median_cycles": {"prologue": int(np.median(d[:, 0])), "stages": int(np.median(d[:, 1])),
                             "epilogue": int(np.median(d[:, 2])), "total": int(np.median(total))},
           "outside_stage_loop_share": round(float(np.median((d[:, 0] + d[:, 2]) / total)), 4),
           "median_gap_to_next_wg_same_cu": int(np.median(gaps)) if gaps else None,
           "gap_share": round(float(np.median(gaps) / np.median(total)), 4) if gaps else None}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
