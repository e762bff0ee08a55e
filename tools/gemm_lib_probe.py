"""How fast would the library GEMM (torch.matmul -> hipBLASLt on ROCm) run the split ViT
GEMM shapes?  (GPU box probe; bf16 in / bf16 out, f32 accumulation.)

The split forward computes A_hi W_hi + A_lo W_hi + A_hi W_lo: as library calls that is
[A_hi | A_lo] (K = 2 K0) against [W_hi ; W_hi] plus A_hi (K0) against W_lo.  Prints ms and
TFLOP/s (3 K0 products counted) per shape at the bench's 246-frame batch (M = 130,380)."""
import json

import torch


def main():
    dev = torch.device("cuda")
    M = 246 * 530
    res = {}
    for name, N, K0 in (("qkv", 2304, 768), ("proj", 768, 768), ("fc1", 3072, 768), ("fc2", 768, 3072)):
        a2 = torch.randn(M, 2 * K0, device=dev).to(torch.bfloat16)
        w2 = torch.randn(2 * K0, N, device=dev).to(torch.bfloat16)
        a1 = a2[:, :K0]
        w1 = torch.randn(K0, N, device=dev).to(torch.bfloat16)
        for _ in range(3):
            c = a2 @ w2
            c = torch.addmm(c, a1, w1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 10
        e0.record()
        for _ in range(it):
            c = a2 @ w2
            c = torch.addmm(c, a1, w1)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        res[name] = {"ms": round(ms, 3), "tflops": round(2.0 * M * N * 3 * K0 / (ms * 1e9), 1)}
        del a2, w2, w1, c
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
