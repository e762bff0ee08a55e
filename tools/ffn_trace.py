"""Phase timeline of the fused LightGlue block tail (lg_ffn.hip) from a -DMLG_FFN_TRACE=1
build (GPU box tool, run through tools/ab_run.py --lib-dir <trace build>): one launch on
seeded inputs, then per workgroup the s_memtime stamps at its phase boundaries and the
CU it ran on (HW_ID / XCC_ID).  Prints the median cycles of each phase and, for the
workgroups that shared a CU, how their phases lined up in time.

    python tools/ab_run.py --lib-dir ab_ffnt tools/ffn_trace.py [--tokens 2097152]
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

PHASES = ["load", "msg_gemm", "msg_epilogue", "ffn1_gemm", "ln_stats", "gelu", "ffn2_gemm", "ffn2_stage",
          "residual"]
MEM = {0, 8}  # phase indices that move HBM bytes (tile load, residual row pass)


def p(t):
    return ctypes.c_void_p(t.data_ptr())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=1 << 21)
    a = ap.parse_args()
    L = _native.lib()
    dev = torch.device("cuda:0")
    M = a.tokens
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device=dev).manual_seed(0)
    bf = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.05).to(torch.bfloat16)  # noqa: E731
    f32 = lambda *s: torch.randn(*s, device=dev, generator=g) * 0.1  # noqa: E731
    cat = (torch.randn(M, 512, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    ctx = (torch.randn(M, 256, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    X = torch.randn(M, 256, device=dev, generator=g)
    Wo, bo, W1, b1, W2, b2 = bf(256 * 256), f32(256), bf(512 * 512), f32(512), bf(256 * 512), f32(256)
    lng, lnb = f32(512) + 1, f32(512)
    ffn = lambda: L.mlg_op_lg_ffn(p(ctx), p(X), p(cat), 512, M, p(Wo), p(bo), p(W1), p(b1),  # noqa: E731
                                  p(lng), p(lnb), p(W2), p(b2), st)
    for _ in range(3):
        assert ffn() == 0
    torch.cuda.synchronize()
    nwg = (M + 63) // 64
    buf = np.zeros((65536, 12), np.uint64)
    rc = L.mlg_dbg_ffn_trace(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
    if rc != 0:
        raise SystemExit(f"mlg_dbg_ffn_trace returned {rc}: not a -DMLG_FFN_TRACE=1 build")
    tr = buf[:min(nwg, 65536)].astype(np.int64)
    t = tr[:, :10]
    dur = np.diff(t, axis=1)  # [wg, 9]
    hw, xcc = tr[:, 10], tr[:, 11]
    cu_key = (xcc & 15) * 4096 + ((hw >> 13) & 7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 15)
    res = {"tokens": M, "workgroups": int(len(t)), "cus_seen": int(len(np.unique(cu_key))),
           "median_cycles": {PHASES[i]: int(np.median(dur[:, i])) for i in range(9)},
           "median_tile_cycles": int(np.median(t[:, 9] - t[:, 0]))}
    # co-residency: per CU, workgroups sorted by start; for each workgroup the fraction of
    # its memory-phase cycles during which the other resident workgroup was also in a
    # memory phase (1 = lockstep, ~share of memory time = independent)
    both, mine, starts_gap = 0, 0, []
    for k in np.unique(cu_key):
        idx = np.flatnonzero(cu_key == k)
        idx = idx[np.argsort(t[idx, 0])]
        for n, i in enumerate(idx):
            near = [ii for ii in idx[max(0, n - 3):n + 4] if ii != i]
            for j in MEM:
                s, e = int(t[i, j]), int(t[i, j + 1])
                mine += e - s
                for ii in near:
                    for j2 in MEM:
                        s2, e2 = int(t[ii, j2]), int(t[ii, j2 + 1])
                        both += max(0, min(e, e2) - max(s, s2))
        st0 = np.sort(t[idx, 0])
        if len(st0) > 1:
            starts_gap.extend(np.diff(st0).tolist())
    res["memory_overlap_with_coresident"] = round(both / max(mine, 1), 3)
    res["memory_share_of_tile"] = round(float(np.median(dur[:, 0] + dur[:, 8]) / np.median(t[:, 9] - t[:, 0])), 3)
    res["median_start_gap_same_cu"] = int(np.median(starts_gap)) if starts_gap else None
    print(json.dumps(res), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"ffn_trace_{M}.npz"), trace=tr)


if __name__ == "__main__":
    main()
