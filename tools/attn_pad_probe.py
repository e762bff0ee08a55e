"""Does k_attention_varlen (ViT layout via mlg_op_attention) read key / query pad rows or
V^T pad columns?  Same valid data, pads zero vs large vs NaN; report max |dO|."""
import json
import sys

import torch

sys.path.insert(0, "multi-level-indoor-slam_amd")
from mlgate import _native  # noqa: E402

dev = torch.device("cuda:0")
P = lambda t: t.data_ptr()  # noqa: E731
S = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
B, T = 3, 530
Tpad = (T + 63) // 64 * 64
g = torch.Generator().manual_seed(0)
q, k, v = (torch.randn(12, B, T, 64, generator=g) * 1.5 for _ in range(3))


def run(kpad=None, qpad=None, vpad=None):
    Qd = torch.zeros(12, B, Tpad, 64)
    Kd = torch.zeros(12, B, Tpad, 64)
    Vp = torch.zeros(12, B, Tpad, 64)
    Qd[:, :, :T], Kd[:, :, :T], Vp[:, :, :T] = q, k, v
    if kpad is not None:
        Kd[:, :, T:] = kpad
    if qpad is not None:
        Qd[:, :, T:] = qpad
    if vpad is not None:
        Vp[:, :, T:] = vpad
    Qd, Kd = Qd.to(torch.bfloat16).to(dev), Kd.to(torch.bfloat16).to(dev)
    Vt = Vp.to(torch.bfloat16).reshape(12, B * Tpad // 64, 64, 64).transpose(-1, -2).contiguous().to(dev)
    O = torch.full((B * T, 768), float("nan"), dtype=torch.bfloat16, device=dev)
    tw = torch.empty(5 * B, dtype=torch.int32, device=dev)
    _native.check(_native.lib().mlg_op_attention(P(Qd), P(Kd), P(Vt), P(O), B, T, Tpad, P(tw), S()), "attn")
    torch.cuda.synchronize()
    return O.float().cpu()


ref = run()
res = {"nan_in_ref": bool(torch.isnan(ref).any())}
for name, kw in (("k_big", dict(kpad=1e4)), ("k_nan", dict(kpad=float("nan"))), ("q_nan", dict(qpad=float("nan"))),
                 ("v_big", dict(vpad=1e4)), ("again", {})):
    o = run(**kw)
    d = (o - ref).abs()
    res[name] = {"max_abs": float(torch.nan_to_num(d, nan=1e30).max()), "rows": int((d.nan_to_num(1e30) > 0).any(1).sum())}
print(json.dumps(res))
