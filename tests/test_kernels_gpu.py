"""Op-level parity of the HIP kernels (called through the C ABI) against float32
PyTorch references of the same op and against the CPU oracle.  GPU only."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mlgate import _native

pytestmark = pytest.mark.gpu


def P(t):
    return ctypes.c_void_p(t.data_ptr())


def S(dev):
    return _native.stream_of(dev)


def bf16_bits(x):
    return x.to(torch.bfloat16).contiguous()


def rel_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (1060, 256, 768), (530, 3072, 768), (777, 768, 3072),
                                   (33920 - 17, 2304, 768), (129, 256, 192)])
def test_gemm_f32out(dev, M, N, K, variant):
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(dev)
    W = torch.randn(N, K, generator=g).to(dev)
    Ab, Wb = bf16_bits(A), bf16_bits(W)
    C = torch.full((M, N), float("nan"), device=dev)
    _native.check(_native.lib().mlg_op_gemm_f32out_variant(variant, P(Ab), P(Wb), P(C), M, N, K, S(dev)), "gemm")
    ref = Ab.float().cpu() @ Wb.float().cpu().T
    torch.cuda.synchronize()
    assert torch.isfinite(C).all()
    assert rel_err(C.cpu(), ref) < 1e-5


def test_gemm_asymmetric_identity(dev):
    """A = I with asymmetric W catches a transposed C-write (guide §3)."""
    M = N = 128
    K = 128
    A = torch.eye(M, K, device=dev)
    W = (torch.arange(N, device=dev)[:, None] * 1000 + torch.arange(K, device=dev)[None, :]).float() / 256.0
    Ab, Wb = bf16_bits(A), bf16_bits(W)
    C = torch.empty(M, N, device=dev)
    _native.check(_native.lib().mlg_op_gemm_f32out(P(Ab), P(Wb), P(C), M, N, K, S(dev)), "gemm")
    torch.cuda.synchronize()
    assert torch.equal(C.cpu(), Wb.float().cpu().T)


def test_gemm_gelu_and_residual(dev):
    M, N, K = 600, 384, 768
    g = torch.Generator().manual_seed(3)
    A = bf16_bits(torch.randn(M, K, generator=g).to(dev) * 0.5)
    W = bf16_bits(torch.randn(N, K, generator=g).to(dev) * 0.05)
    b = torch.randn(N, generator=g).to(dev) * 0.1
    gam = torch.rand(N, generator=g).to(dev)
    H = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    _native.check(_native.lib().mlg_op_gemm_bias_gelu(P(A), P(W), P(b), P(H), M, N, K, S(dev)), "gelu")
    ref = F.gelu(A.float().cpu() @ W.float().cpu().T + b.cpu())
    torch.cuda.synchronize()
    assert rel_err(H.float().cpu(), ref) < 5e-3
    X0 = torch.randn(M, N, generator=g).to(dev)
    X = X0.clone()
    _native.check(_native.lib().mlg_op_gemm_residual(P(A), P(W), P(b), P(gam), P(X), M, N, K, S(dev)), "res")
    ref = X0.cpu() + gam.cpu() * (A.float().cpu() @ W.float().cpu().T + b.cpu())
    torch.cuda.synchronize()
    assert rel_err(X.cpu(), ref) < 1e-5


def test_gemm_rejects_bad_shapes(dev):
    A = torch.zeros(64, 96, dtype=torch.bfloat16, device=dev)
    W = torch.zeros(128, 96, dtype=torch.bfloat16, device=dev)
    C = torch.zeros(64, 128, device=dev)
    assert _native.lib().mlg_op_gemm_f32out(P(A), P(W), P(C), 64, 128, 96, S(dev)) == -1  # K % 64
    assert _native.lib().mlg_op_gemm_f32out(P(A), P(W), P(C), 64, 100, 64, S(dev)) == -1  # N % 128


def test_layernorm(dev):
    M = 1061
    g = torch.Generator().manual_seed(5)
    X = (torch.randn(M, 768, generator=g) * 3 + 1).to(dev)
    w = (1 + 0.1 * torch.randn(768, generator=g)).to(dev)
    b = (0.1 * torch.randn(768, generator=g)).to(dev)
    Y = torch.empty(M, 768, dtype=torch.bfloat16, device=dev)
    _native.check(_native.lib().mlg_op_layernorm_bf16(P(X), P(w), P(b), P(Y), M, S(dev)), "ln")
    ref = F.layer_norm(X.cpu(), (768,), w.cpu(), b.cpu(), eps=1e-6)
    torch.cuda.synchronize()
    assert rel_err(Y.float().cpu(), ref) < 4e-3


@pytest.mark.parametrize("B,T", [(2, 530), (1, 64), (3, 197), (1, 1370)])
def test_attention(dev, B, T):
    Tpad = (T + 63) // 64 * 64
    g = torch.Generator().manual_seed(T)
    q, k, v = (torch.randn(B, 12, T, 64, generator=g) * 1.5 for _ in range(3))
    q, k, v = (bf16_bits(x) for x in (q, k, v))
    # head-major segments (image b at rows b * Tpad of each head), V^T tiled per 64 keys
    Qd = torch.zeros(12, B, Tpad, 64, dtype=torch.bfloat16)
    Kd = torch.zeros(12, B, Tpad, 64, dtype=torch.bfloat16)
    Vp = torch.zeros(12, B, Tpad, 64, dtype=torch.bfloat16)
    Qd[:, :, :T] = q.transpose(0, 1)
    Kd[:, :, :T] = k.transpose(0, 1)
    Vp[:, :, :T] = v.transpose(0, 1)
    Vt = Vp.reshape(12, B * Tpad // 64, 64, 64).transpose(-1, -2).contiguous()
    Qd, Kd, Vt = Qd.to(dev), Kd.to(dev), Vt.to(dev)
    O = torch.empty(B * T, 768, dtype=torch.bfloat16, device=dev)
    tw = torch.empty(5 * B, dtype=torch.int32, device=dev)
    _native.check(_native.lib().mlg_op_attention(P(Qd), P(Kd), P(Vt), P(O), B, T, Tpad, P(tw), S(dev)), "attn")
    a = ((q.float() * 0.125) @ k.float().transpose(-1, -2)).softmax(-1)
    ref = (a @ v.float()).transpose(1, 2).reshape(B * T, 768)
    torch.cuda.synchronize()
    assert rel_err(O.float().cpu(), ref) < 1e-2


def _patches_ref(img, S_=322):
    from oracle import vit as ovit
    x = ovit.preprocess(img, S_)  # [1, 3, S, S] f32
    g = S_ // 14
    p = x.reshape(3, g, 14, g, 14).permute(1, 3, 0, 2, 4).reshape(g * g, 588)
    return p


@pytest.mark.parametrize("shape", [(480, 640, 3), (540, 720, 3), (480, 640, 4), (480, 640), (77, 100, 3)])
def test_preprocess_bit_exact(dev, shape):
    rng = np.random.default_rng(sum(shape))
    imgs = rng.integers(0, 256, (2,) + shape, dtype=np.uint8)
    fr = torch.from_numpy(imgs).to(dev)
    H, W = shape[:2]
    C = 1 if len(shape) == 2 else shape[2]
    from mlgate.vit import PATCH_K
    out = torch.empty(2 * 529, PATCH_K, dtype=torch.bfloat16, device=dev)
    _native.check(_native.lib().mlg_op_preprocess_patches(P(fr), 2, H, W, C, H * W * C, 322, P(out), S(dev)),
                  "prep")
    torch.cuda.synchronize()
    out = out.cpu()
    for b in range(2):
        ref = _patches_ref(imgs[b]).to(torch.bfloat16)
        got = out[b * 529:(b + 1) * 529]
        assert torch.equal(got[:, :588].view(torch.int16), ref.view(torch.int16))
        assert torch.count_nonzero(got[:, 588:].float()) == 0


@pytest.mark.parametrize("lens", [(64, 70), (1, 200, 3, 129), (700, 650, 2048, 1900), (300, 17)])
def test_attention_varlen(dev, lens):
    """LightGlue's ragged self / cross attention (k_attention_varlen) vs float32 softmax."""
    H = 4
    lens = np.array(lens)
    offs = np.concatenate([[0], np.cumsum((lens + 63) // 64 * 64)])
    Npad = int(offs[-1])
    g = torch.Generator().manual_seed(int(lens.sum()))
    Q = bf16_bits(torch.randn(H, Npad, 64, generator=g) * 1.5)
    K = bf16_bits(torch.randn(H, Npad, 64, generator=g) * 1.5)
    V = bf16_bits(torch.randn(H, Npad, 64, generator=g))
    Vt = V.view(H, Npad // 64, 64, 64).transpose(2, 3).contiguous()
    tasks, outs = [], []
    for i in range(len(lens)):  # self, then cross with the next segment
        j = (i + 1) % len(lens)
        tasks += [(offs[i], lens[i], offs[i], lens[i])]
        tasks += [(offs[i], lens[i], offs[j], lens[j])]
    O = torch.zeros(2, Npad, H * 64, dtype=torch.bfloat16, device=dev)
    L = _native.lib()
    Qd, Kd, Vd = Q.to(dev), K.to(dev), Vt.to(dev)  # kept alive until the launches have run
    for kind in range(2):
        T = torch.tensor(np.array(tasks[kind::2], np.int32), device=dev)
        OO = torch.tensor(np.array([t[0] for t in tasks[kind::2]], np.int32), device=dev)
        _native.check(L.mlg_op_attention_varlen(P(Qd), P(Kd), P(Vd), P(O[kind]), H * 64, Npad, H, P(T), P(OO),
                                                len(T), int(lens.max()), S(dev)), "attn varlen")
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    O = O.float().cpu()
    for n, (qo, ql, ko, kl) in enumerate(tasks):
        q, k, v = Q[:, qo:qo + ql].float(), K[:, ko:ko + kl].float(), V[:, ko:ko + kl].float()
        ref = (torch.softmax(q @ k.transpose(1, 2) / 8.0, -1) @ v).transpose(0, 1).reshape(ql, H * 64)
        got = O[n % 2, qo:qo + ql]
        assert rel_err(got, ref) < 1e-2, (n, rel_err(got, ref))


@pytest.mark.parametrize("shape", [("vit", 123, 530), ("ragged", 200, 2048), ("ragged", 369, 530)])
def test_attention_run_to_run_exact(dev, shape):
    """k_attention_varlen gives the same bits on every run of the same inputs, at loads that
    fill the chip (regression: the row max's inline asm read MFMA results without the XDL
    wait states, and up to ~0.1 % of rows differed run to run; tools/attn_det_probe.py)."""
    kind, n, T = shape
    H = 12 if kind == "vit" else 4
    Tp = (T + 63) // 64 * 64
    g = torch.Generator(device=dev).manual_seed(T)
    Q = (torch.randn(H, n, Tp, 64, generator=g, device=dev) * 1.5).to(torch.bfloat16)
    K = (torch.randn(H, n, Tp, 64, generator=g, device=dev) * 1.5).to(torch.bfloat16)
    V = torch.randn(H, n, Tp, 64, generator=g, device=dev) * 1.5
    V[:, :, T:] = 0
    Vt = V.to(torch.bfloat16).reshape(H, n * Tp // 64, 64, 64).transpose(-1, -2).contiguous()
    L = _native.lib()
    outs = []
    if kind == "vit":
        tw = torch.empty(5 * n, dtype=torch.int32, device=dev)
        for _ in range(3):
            O = torch.empty(n * T, 768, dtype=torch.bfloat16, device=dev)
            _native.check(L.mlg_op_attention(P(Q), P(K), P(Vt), P(O), n, T, Tp, P(tw), S(dev)), "attn")
            torch.cuda.synchronize()
            outs.append(O)
    else:
        tasks = torch.tensor([[i * Tp, T, i * Tp, T] for i in range(n)], dtype=torch.int32, device=dev)
        oo = torch.tensor([i * Tp for i in range(n)], dtype=torch.int32, device=dev)
        for _ in range(3):
            O = torch.zeros(n * Tp, H * 64, dtype=torch.bfloat16, device=dev)
            _native.check(L.mlg_op_attention_varlen(P(Q), P(K), P(Vt), P(O), H * 64, n * Tp, H, P(tasks), P(oo), n, T,
                                                    S(dev)), "attn varlen")
            torch.cuda.synchronize()
            outs.append(O)
    for o in outs[1:]:
        assert torch.equal(o.view(torch.int16), outs[0].view(torch.int16))


@pytest.mark.parametrize("M", [192, 1000, 128])
def test_lg_ffn_fused(dev, M):
    """Fused LightGlue block tail (lg_ffn.hip) vs float32 torch on the same bf16 operands."""
    g = torch.Generator().manual_seed(M)
    w = {"Wout": (256, 256), "Wf1": (512, 512), "Wf2": (256, 512)}
    W = {k: bf16_bits(torch.randn(*s, generator=g) / s[1] ** 0.5) for k, s in w.items()}
    b = {k: torch.randn(n, generator=g) * 0.1 for k, n in (("bout", 256), ("bf1", 512), ("bf2", 256))}
    ln_g, ln_b = 1 + 0.1 * torch.randn(512, generator=g), 0.1 * torch.randn(512, generator=g)
    X = torch.randn(M, 256, generator=g)
    ctx = bf16_bits(torch.randn(M, 256, generator=g))
    Xd = X.to(dev)
    xc = torch.zeros(M, 512, dtype=torch.bfloat16, device=dev)
    xc[:, :256] = bf16_bits(X).to(dev)  # the bf16 copy of x the previous block wrote
    from mlgate.lightglue import pack_kstep
    dW = {k: torch.from_numpy(pack_kstep(v.float().numpy())).to(torch.bfloat16).to(dev) for k, v in W.items()}
    db = {k: v.to(dev) for k, v in b.items()}
    gd, bd = ln_g.to(dev), ln_b.to(dev)
    ctxd = ctx.to(dev)
    _native.check(_native.lib().mlg_op_lg_ffn(P(ctxd), P(Xd), P(xc), 512, M, P(dW["Wout"]), P(db["bout"]),
                                              P(dW["Wf1"]), P(db["bf1"]), P(gd), P(bd), P(dW["Wf2"]), P(db["bf2"]),
                                              S(dev)), "lg_ffn")
    torch.cuda.synchronize()
    msg = bf16_bits(ctx.float() @ W["Wout"].float().T + b["bout"]).float()
    cat = torch.cat([bf16_bits(X).float(), msg], -1)
    h = cat @ W["Wf1"].float().T + b["bf1"]
    h = bf16_bits(F.gelu(F.layer_norm(h, (512,), ln_g, ln_b))).float()
    ref = X + h @ W["Wf2"].float().T + b["bf2"]
    got = Xd.cpu()
    assert rel_err(got - X, ref - X) < 1e-2
    assert torch.equal(xc[:, :256].cpu(), bf16_bits(got))


@pytest.mark.parametrize("self_block", [True, False])
def test_lg_proj(dev, self_block):
    """LightGlue projections (lg_proj.hip) vs float32 torch on the same bf16 operands:
    q / k (+ rotary) in [4][Npad][64], v in the tiled V^T; dead rows zero."""
    from mlgate.lightglue import pack_kstep, pack_rotary
    Npad, H = 192, 4
    N = 768 if self_block else 512
    g = torch.Generator().manual_seed(N)
    x = bf16_bits(torch.randn(Npad, 256, generator=g))
    W = bf16_bits(torch.randn(N, 256, generator=g) / 16)
    b = torch.randn(N, generator=g) * 0.1
    ang = torch.rand(Npad, 32, generator=g) * 6.3
    ec, es = torch.cos(ang), torch.sin(ang)
    live = (torch.rand(Npad, generator=g) > 0.2).to(torch.uint8)
    xc = torch.zeros(Npad, 512, dtype=torch.bfloat16)
    xc[:, :256] = x
    d = {k: v.to(dev) for k, v in dict(xc=xc, b=b, ef=pack_rotary(ec, es), live=live).items()}
    Wd = torch.from_numpy(pack_kstep(W.float().numpy())).to(torch.bfloat16).to(dev)
    Q = torch.full((H, Npad, 64), 7.0, dtype=torch.bfloat16, device=dev)
    K = torch.full((H, Npad, 64), 7.0, dtype=torch.bfloat16, device=dev)
    Vt = torch.full((H, Npad // 64, 64, 64), 7.0, dtype=torch.bfloat16, device=dev)
    _native.check(_native.lib().mlg_op_lg_proj(int(self_block), P(d["xc"]), 512, P(Wd), P(d["b"]), P(d["ef"]),
                                               None, P(d["live"]), P(Q), P(K), P(Vt), Npad, S(dev)), "lg_proj")
    torch.cuda.synchronize()
    y = x.float() @ W.float().T + b  # [Npad, N]
    heads = lambda t: t.view(Npad, H, 64).transpose(0, 1)  # noqa: E731
    m = live.bool()[None, :, None]
    if self_block:
        c2, s2 = ec.repeat_interleave(2, -1), es.repeat_interleave(2, -1)
        rot = lambda t: t * c2 + torch.stack([-t[..., 1::2], t[..., 0::2]], -1).flatten(-2) * s2  # noqa: E731
        refq, refk, refv = rot(heads(y[:, :256])), rot(heads(y[:, 256:512])), heads(y[:, 512:])
        assert rel_err(K.float().cpu() * m, refk * m) < 1e-2
        assert torch.all(K.float().cpu()[~m.expand_as(refk)] == 0)
    else:
        refq, refv = heads(y[:, :256]), heads(y[:, 256:])
    assert rel_err(Q.float().cpu() * m, refq * m) < 1e-2
    assert torch.all(Q.float().cpu()[~m.expand_as(refq)] == 0)
    v = Vt.float().cpu().transpose(2, 3).reshape(H, Npad, 64)
    assert rel_err(v * m, refv * m) < 1e-2
    assert torch.all(v[~m.expand_as(refv)] == 0)


def test_lightglue_kernels_deterministic(dev):
    """The LightGlue projection, attention and fused block-tail kernels are bit-for-bit
    deterministic run to run on the same inputs (no races, no order-dependent sums)."""
    from mlgate.lightglue import pack_kstep, pack_rotary
    L = _native.lib()
    Npad, H = 8192, 4
    g = torch.Generator().manual_seed(11)
    xc = torch.zeros(Npad, 512, dtype=torch.bfloat16)
    xc[:, :256] = bf16_bits(torch.randn(Npad, 256, generator=g))
    X = xc[:, :256].float().clone()
    W = torch.from_numpy(pack_kstep((torch.randn(768, 256, generator=g) / 16).numpy())).to(torch.bfloat16)
    b = torch.randn(768, generator=g) * 0.1
    ang = torch.rand(Npad, 32, generator=g) * 6.3
    live = (torch.rand(Npad, generator=g) > 0.1).to(torch.uint8)
    d = {k: v.to(dev) for k, v in dict(xc=xc, W=W, b=b, ef=pack_rotary(torch.cos(ang), torch.sin(ang)),
                                       live=live).items()}
    outs = []
    for _ in range(3):
        Q = torch.zeros(H, Npad, 64, dtype=torch.bfloat16, device=dev)
        K = torch.zeros_like(Q)
        Vt = torch.zeros(H, Npad // 64, 64, 64, dtype=torch.bfloat16, device=dev)
        _native.check(L.mlg_op_lg_proj(1, P(d["xc"]), 512, P(d["W"]), P(d["b"]), P(d["ef"]), None,
                                       P(d["live"]), P(Q), P(K), P(Vt), Npad, S(dev)), "proj")
        tasks = torch.tensor([[s, 2048, s, 2048] for s in range(0, Npad, 2048)], dtype=torch.int32, device=dev)
        oo = tasks[:, 0].contiguous()
        O = torch.zeros(Npad, 256, dtype=torch.bfloat16, device=dev)
        _native.check(L.mlg_op_attention_varlen(P(Q), P(K), P(Vt), P(O), 256, Npad, H, P(tasks), P(oo), len(tasks),
                                                2048, S(dev)), "attn")
        Xd, xcd = X.to(dev), d["xc"].clone()
        w = {k: torch.from_numpy(pack_kstep((torch.randn(*s, generator=torch.Generator().manual_seed(5)) / 16)
                                            .numpy())).to(torch.bfloat16).to(dev)
             for k, s in (("o", (256, 256)), ("f1", (512, 512)), ("f2", (256, 512)))}
        vec = {n: torch.full((n,), 0.01, device=dev) for n in (256, 512)}
        _native.check(L.mlg_op_lg_ffn(P(O), P(Xd), P(xcd), 512, Npad, P(w["o"]), P(vec[256]), P(w["f1"]), P(vec[512]),
                                      P(torch.ones(512, device=dev)), P(vec[512]), P(w["f2"]), P(vec[256]), S(dev)),
                      "ffn")
        torch.cuda.synchronize()
        outs.append((Q.cpu(), K.cpu(), Vt.cpu(), O.cpu(), Xd.cpu()))
    bad = [name for o in outs[1:] for name, a, r in zip("QKVOX", o, outs[0]) if not torch.equal(a, r)]
    assert not bad, bad
