"""k_attention_varlen determinism across shapes through a library directory given on the
command line: three runs on identical inputs (random pad rows), bitwise comparison.
Configs: (B, T) of the ViT op (12 heads, ldo 768) and (ntasks, len, heads) of the ragged op."""
import ctypes
import json
import os
import sys

import torch

lib = ctypes.CDLL(os.path.join(sys.argv[1], "libmlgate.so"))
vp, ci = ctypes.c_void_p, ctypes.c_int
lib.mlg_op_attention.argtypes = [vp, vp, vp, vp, ci, ci, ci, vp, vp]
lib.mlg_op_attention_varlen.argtypes = [vp, vp, vp, vp, ci, ci, ci, vp, vp, ci, ci, vp]
dev = torch.device("cuda:0")
stream = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731


def inputs(H, B, T, Tpad, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    Q = (torch.randn(H, B, Tpad, 64, generator=g, device=dev) * 1.5).to(torch.bfloat16)
    K = (torch.randn(H, B, Tpad, 64, generator=g, device=dev) * 1.5).to(torch.bfloat16)
    V = torch.randn(H, B, Tpad, 64, generator=g, device=dev) * 1.5
    V[:, :, T:] = 0
    Vt = V.to(torch.bfloat16).reshape(H, B * Tpad // 64, 64, 64).transpose(-1, -2).contiguous()
    return Q, K, Vt


def vit(B, T):
    Tpad = (T + 63) // 64 * 64
    Q, K, Vt = inputs(12, B, T, Tpad)
    tw = torch.empty(5 * B, dtype=torch.int32, device=dev)
    outs = []
    for _ in range(3):
        O = torch.full((B * T, 768), float("nan"), dtype=torch.bfloat16, device=dev)
        assert lib.mlg_op_attention(Q.data_ptr(), K.data_ptr(), Vt.data_ptr(), O.data_ptr(), B, T, Tpad, tw.data_ptr(),
                                    stream()) == 0
        torch.cuda.synchronize()
        outs.append(O.float())
    return outs


def ragged(n, L, H):
    Lp = (L + 63) // 64 * 64
    Q, K, Vt = inputs(H, n, L, Lp)
    tasks = torch.tensor([[i * Lp, L, i * Lp, L] for i in range(n)], dtype=torch.int32, device=dev)
    oo = torch.tensor([i * Lp for i in range(n)], dtype=torch.int32, device=dev)
    outs = []
    for _ in range(3):
        O = torch.zeros((n * Lp, H * 64), dtype=torch.bfloat16, device=dev)
        assert lib.mlg_op_attention_varlen(Q.data_ptr(), K.data_ptr(), Vt.data_ptr(), O.data_ptr(), H * 64, n * Lp, H,
                                           tasks.data_ptr(), oo.data_ptr(), n, L, stream()) == 0
        torch.cuda.synchronize()
        outs.append(O.float())
    return outs


def cmp(outs):
    r = {}
    for i in (1, 2):
        d = (outs[i] - outs[0]).abs().nan_to_num(1e30)
        r[f"run{i}"] = int((d > 0).any(1).sum())
    r["nan"] = bool(torch.isnan(outs[0]).any())
    return r


res = {}
for B, T in ((123, 530), (123, 512), (123, 576), (123, 1000), (3, 530), (40, 530)):
    res[f"vit_B{B}_T{T}"] = cmp(vit(B, T))
for n, L, H in ((369, 530, 4), (123, 530, 12), (200, 2048, 4), (400, 1000, 4)):
    res[f"ragged_n{n}_L{L}_H{H}"] = cmp(ragged(n, L, H))
print(json.dumps(res))
