"""Which LightGlue kernel gives co-scheduling dependent results, and why?  (GPU box tool.)

    python tools/ffn_interference.py [--rows 65536] [--repeats 6]

For each victim kernel (fused block tail k_lg_ffn, projection k_lg_proj_res, ragged
attention k_attention_varlen) on fixed seeded inputs through the op-level C ABI:

  alone      the same launch repeated on one stream;
  lds        each launch preceded by a kernel filling every CU's LDS with pattern A, then
             with pattern B (mlg_dbg_fill_lds): differences = reads of LDS never written;
  regs       the same with every SIMD's VGPRs / AGPRs (mlg_dbg_fill_regs);
  with_X     the launch repeated while a second thread keeps kernel X (ffn, proj, attn,
             a torch bf16 matmul) busy on its own buffers and stream;

and prints, per (victim, condition), the number of runs whose output differs from the
first alone run and the fraction of differing 64-row tiles."""
import argparse
import json
import os
import sys
import threading

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
sys.path.insert(0, ROOT)

from mlgate import _native  # noqa: E402
from mlgate.lightglue import pack_kstep  # noqa: E402

P = _native.ptr
H = 4


def bf16(t):
    return t.to(torch.bfloat16)


class Case:
    """One set of LightGlue-shaped inputs and the three kernels on them."""

    def __init__(self, rows, dev, seed):
        g = torch.Generator().manual_seed(seed)
        self.rows, self.dev = rows, dev
        xc = torch.zeros(rows, 512, dtype=torch.bfloat16)
        xc[:, :256] = bf16(torch.randn(rows, 256, generator=g))
        self.xc0 = xc.to(dev)
        self.X0 = xc[:, :256].float().to(dev)
        self.W = bf16(torch.from_numpy(pack_kstep((torch.randn(768, 256, generator=g) / 16).numpy()))).to(dev)
        self.b = (torch.randn(768, generator=g) * 0.1).to(dev)
        ang = torch.rand(rows, 32, generator=g) * 6.3
        from mlgate.lightglue import pack_rotary
        self.ec, self.es = pack_rotary(torch.cos(ang), torch.sin(ang)).to(dev), None
        self.live = (torch.rand(rows, generator=g) > 0.1).to(torch.uint8).to(dev)
        self.Q = torch.zeros(H, rows, 64, dtype=torch.bfloat16, device=dev)
        self.K = torch.zeros_like(self.Q)
        self.Vt = torch.zeros(H, rows // 64, 64, 64, dtype=torch.bfloat16, device=dev)
        seg = 2048
        self.tasks = torch.tensor([[s, seg, s, seg] for s in range(0, rows, seg)], dtype=torch.int32, device=dev)
        self.oo = self.tasks[:, 0].contiguous()
        self.O = torch.zeros(rows, 256, dtype=torch.bfloat16, device=dev)
        self.ctx = bf16(torch.randn(rows, 256, generator=g) * 0.5).to(dev)
        self.Xd, self.xcd = self.X0.clone(), self.xc0.clone()
        w = {k: bf16(torch.from_numpy(pack_kstep((torch.randn(*s, generator=g) / 16).numpy()))).to(dev)
             for k, s in (("o", (256, 256)), ("f1", (512, 512)), ("f2", (256, 512)))}
        self.w = w
        self.v256 = (torch.randn(256, generator=g) * 0.01).to(dev)
        self.v512 = (torch.randn(512, generator=g) * 0.01).to(dev)
        self.g512 = (1 + torch.randn(512, generator=g) * 0.1).to(dev)
        self.L = _native.lib()

    def proj(self, s):
        _native.check(self.L.mlg_op_lg_proj(1, P(self.xc0), 512, P(self.W), P(self.b), P(self.ec), None,
                                            P(self.live), P(self.Q), P(self.K), P(self.Vt), self.rows,
                                            torch.cuda.current_stream(self.dev).cuda_stream), "proj")
        return torch.cat([self.Q.view(-1), self.K.view(-1), self.Vt.view(-1)])

    def attn(self, s):
        _native.check(self.L.mlg_op_attention_varlen(P(self.Q), P(self.K), P(self.Vt), P(self.O), 256, self.rows, H,
                                                     P(self.tasks), P(self.oo), len(self.tasks), 2048,
                                                     torch.cuda.current_stream(self.dev).cuda_stream), "attn")
        return self.O.view(-1)

    def ffn(self, s):
        self.Xd.copy_(self.X0)
        self.xcd.copy_(self.xc0)
        w = self.w
        _native.check(self.L.mlg_op_lg_ffn(P(self.ctx), P(self.Xd), P(self.xcd), 512, self.rows, P(w["o"]),
                                           P(self.v256), P(w["f1"]), P(self.v512), P(self.g512), P(self.v512),
                                           P(w["f2"]), P(self.v256),
                                           torch.cuda.current_stream(self.dev).cuda_stream), "ffn")
        return self.Xd.view(-1)


def tiles_differing(a, b, rows):
    a = a.view(-1).view(torch.int16 if a.dtype == torch.bfloat16 else torch.int32)
    b = b.view(-1).view(torch.int16 if b.dtype == torch.bfloat16 else torch.int32)
    d = (a != b)
    n = d.numel()
    per_tile = n // (rows // 64)
    return int(d.view(-1, per_tile).any(1).sum().item()) if n % (rows // 64) == 0 else int(d.sum().item())


def describe(o, ref):
    """Where and how much an FFN output (f32 x [rows, 256]) differs from the reference."""
    o, ref = o.view(-1, 256).cpu(), ref.view(-1, 256).cpu()
    d = o != ref
    rows = torch.nonzero(d.any(1)).view(-1)
    cols = d[rows].sum(0)
    ad = (o - ref).abs()[d]
    rel = (ad / ref.abs()[d].clamp(min=1e-30))
    return {"rows": int(len(rows)), "first_rows": rows[:12].tolist(), "tiles": sorted({int(r) // 64 for r in rows})[:12],
            "rows_in_tile": sorted({int(r) % 64 for r in rows})[:64],
            "cols_per_row_max": int(d[rows].sum(1).max()) if len(rows) else 0,
            "col_groups_64": [int(cols[i * 64:(i + 1) * 64].sum()) for i in range(4)],
            "max_abs": float(ad.max()) if len(ad) else 0.0, "median_rel": float(rel.median()) if len(rel) else 0.0,
            "max_rel": float(rel.max()) if len(rel) else 0.0,
            "nan_or_inf": int((~torch.isfinite(o[rows])).sum())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--repeats", type=int, default=6)
    ap.add_argument("--victims", default="ffn,proj,attn")
    ap.add_argument("--partners", default="ffn,proj,attn,matmul")
    ap.add_argument("--analyse", action="store_true", help="describe the FFN differences (rows, columns, size)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    L = _native.lib()
    sink = torch.zeros(256, dtype=torch.int32, device=dev)
    victim = Case(a.rows, dev, 1)
    partner = Case(a.rows, dev, 2)
    victim.proj(None)  # Q / K / V^T for the attention victim
    torch.cuda.synchronize()
    big = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    s0 = torch.cuda.current_stream(dev)
    res = {}
    for vname in a.victims.split(","):
        run = getattr(victim, vname)
        ref = run(None).clone()
        torch.cuda.synchronize()
        out = {}

        def check(tag, outs):
            bad = [tiles_differing(o, ref, a.rows) for o in outs]
            out[tag] = {"runs": len(outs), "runs_differing": sum(1 for x in bad if x), "max_tiles_differing": max(bad),
                        "tiles": a.rows // 64}

        outs = []
        for _ in range(a.repeats):
            outs.append(run(None).clone())
        torch.cuda.synchronize()
        check("alone", outs)
        for kind, fill in (("lds", lambda p: L.mlg_dbg_fill_lds(p, P(sink), s0.cuda_stream)),
                           ("regs", lambda p: L.mlg_dbg_fill_regs(p, s0.cuda_stream))):
            outs = []
            for pat in (0xFFFFFFFF, 0x3F803F80, 0x00000000, 0x7F7F7F7F):
                _native.check(fill(pat), kind)
                outs.append(run(None).clone())
            torch.cuda.synchronize()
            check(kind, outs)
        for pname in a.partners.split(","):
            stop = threading.Event()
            ps = torch.cuda.Stream(dev)

            def loop():
                with torch.cuda.stream(ps):
                    while not stop.is_set():
                        for _ in range(4):
                            if pname == "matmul":
                                torch.matmul(big, big)
                            else:
                                getattr(partner, pname)(None)
                        ps.synchronize()
            th = threading.Thread(target=loop)
            th.start()
            outs = []
            try:
                for _ in range(a.repeats):
                    outs.append(run(None).clone())
                    torch.cuda.synchronize(dev) if False else s0.synchronize()
            finally:
                stop.set()
                th.join()
            check(f"with_{pname}", outs)
            if a.analyse and vname == "ffn":
                out[f"with_{pname}"]["detail"] = [describe(o, ref) for o in outs if not torch.equal(o, ref)][:4]
        res[vname] = out
        print(json.dumps({vname: out}), flush=True)
    print(json.dumps({"summary": res}), flush=True)


if __name__ == "__main__":
    main()
