"""SuperGlue on the GPU (superglue.hip via mlg_superglue) against the torch-fp32
restatement (oracle/superglue.py, bf16 operand emulation) with the same seeded weights
and inputs.

The GNN runs 18 bf16 layers, so the two differ by summation order and bf16 rounding of
the weights; matches are discrete decisions (mutual argmax, exp(score) > 0.2), so the
bar is: >= 95 % of matches identical, scores of common matches within 5e-2 absolute.
Batched and single-pair calls must agree bit for bit; an empty side yields no matches
(magicleap's early exit).  Parity vs the trained magicleap model is unpinned (offline).
"""
import numpy as np
import pytest
import torch

from mlgate.superglue import SuperGlueGPU
from mlgate.weights import superglue_state_dict
from oracle.superglue import Oracle

pytestmark = pytest.mark.gpu
W, H = 640, 480


def feats(rng, m, n, overlap=0.6):
    k0 = np.stack([rng.uniform(0, W, m), rng.uniform(0, H, m)], 1).astype(np.float32)
    d0 = rng.standard_normal((m, 256)).astype(np.float32)
    d0 /= np.linalg.norm(d0, axis=1, keepdims=True)
    no = int(overlap * min(m, n))
    k1 = np.stack([rng.uniform(0, W, n), rng.uniform(0, H, n)], 1).astype(np.float32)
    d1 = rng.standard_normal((n, 256)).astype(np.float32)
    k1[:no] = k0[:no] + rng.normal(0, 2, (no, 2)) + np.array([15, -8])
    d1[:no] = d0[:no] + 0.02 * rng.standard_normal((no, 256))
    d1 /= np.linalg.norm(d1, axis=1, keepdims=True) + 1e-12
    s0 = rng.uniform(0.005, 1.0, m).astype(np.float32)
    s1 = rng.uniform(0.005, 1.0, n).astype(np.float32)
    return k0, s0, d0, k1.astype(np.float32), s1, d1.astype(np.float32)


@pytest.fixture(scope="module")
def sd():
    return superglue_state_dict(0)


@pytest.fixture(scope="module")
def sg(dev, sd):
    return SuperGlueGPU(sd, device=str(dev))


def _run_gpu(sg, cases):
    kmax = max(max(len(c[0]), len(c[3]), 1) for c in cases)
    F = 2 * len(cases)
    kp = torch.zeros(F, kmax, 2)
    sc = torch.zeros(F, kmax)
    ds = torch.zeros(F, kmax, 256)
    counts = []
    for i, (k0, s0, d0, k1, s1, d1) in enumerate(cases):
        for j, (k, s, d) in enumerate(((k0, s0, d0), (k1, s1, d1))):
            kp[2 * i + j, :len(k)] = torch.from_numpy(k)
            sc[2 * i + j, :len(k)] = torch.from_numpy(s)
            ds[2 * i + j, :len(k)] = torch.from_numpy(d)
            counts.append(len(k))
    m, s, n = sg.match_device(kp.to(sg.device), sc.to(sg.device), ds.to(sg.device), counts, np.arange(0, F, 2),
                              np.arange(1, F, 2), W, H)
    m, s, n = m.cpu().numpy(), s.cpu().numpy(), n.cpu().numpy()
    return [(m[p, :n[p]], s[p, :n[p]]) for p in range(len(cases))]


@pytest.mark.parametrize("m,n", [(700, 650), (2048, 1900), (1700, 300), (64, 70), (3, 5)])
def test_superglue_matches_oracle(sg, sd, m, n):
    rng = np.random.default_rng(m + n)
    case = feats(rng, m, n)
    got_m, got_s = _run_gpu(sg, [case])[0]
    rm, rs = Oracle(sd, emulate_bf16=True).match(*case, W, H)
    g = {tuple(x): i for i, x in enumerate(got_m.tolist())}
    r = {tuple(x): i for i, x in enumerate(rm.tolist())}
    common = set(g) & set(r)
    assert len(common) >= 0.95 * max(len(g), len(r)) - 1, (len(common), len(g), len(r))
    if common:
        gi = np.array([g[c] for c in common], int)
        ri = np.array([r[c] for c in common], int)
        assert np.abs(got_s[gi] - rs[ri]).max() < 5e-2
    if len(got_m):
        assert np.all(got_s > 0.2) and np.all(np.diff(got_m[:, 0]) > 0)
    if m >= 64:
        assert len(got_m) >= 0.5 * int(0.6 * min(m, n))  # the shared points are found


@pytest.mark.parametrize("m,n", [(700, 650), (2048, 1900)])
def test_superglue_against_fp32_reference(sg, sd, m, n):
    """The GPU SuperGlue (bf16 GNN, f32 Sinkhorn) against the float32 restatement
    (oracle/superglue.py with emulate_bf16=False): match-set overlap and score error."""
    rng = np.random.default_rng(7 * m + n)
    case = feats(rng, m, n)
    got_m, got_s = _run_gpu(sg, [case])[0]
    rm, rs = Oracle(sd, emulate_bf16=False).match(*case, W, H)
    g = {tuple(x): i for i, x in enumerate(got_m.tolist())}
    r = {tuple(x): i for i, x in enumerate(rm.tolist())}
    common = set(g) & set(r)
    overlap = len(common) / max(len(g), len(r), 1)
    err = 0.0
    if common:
        gi = np.array([g[c] for c in common], int)
        ri = np.array([r[c] for c in common], int)
        err = float(np.abs(got_s[gi] - rs[ri]).max())
    print(f"fp32 SuperGlue {m}x{n}: {len(g)} vs {len(r)} matches, overlap {overlap:.4f}, max score err {err:.4f}")
    assert len(r) > 50 and overlap >= 0.99  # measured 1.0000 / 1.0000 (profiles/r03ae_tolerances.log)
    assert err < 1e-2  # measured 0.0012 / 0.0017


def test_superglue_batch_equals_single_and_empty_sides(sg):
    rng = np.random.default_rng(11)
    cases = [feats(rng, 900, 800), feats(rng, 130, 1200), feats(rng, 400, 410)]
    e = feats(rng, 50, 60)
    empty = (e[0], e[1], e[2], e[3][:0], e[4][:0], e[5][:0])
    batch = _run_gpu(sg, cases[:2] + [empty] + cases[2:])
    singles = [_run_gpu(sg, [c])[0] for c in cases]
    for (bm, bs), (sm, ss) in zip(batch[:2] + batch[3:], singles):
        assert np.array_equal(bm, sm) and np.array_equal(bs, ss)
    assert len(batch[2][0]) == 0
    again = _run_gpu(sg, cases[:2] + [empty] + cases[2:])
    for (a, sa), (b, sb) in zip(batch, again):
        assert np.array_equal(a, b) and np.array_equal(sa, sb)


def test_superglue_verifier_native(dev, monkeypatch):
    """verify.SuperGlue with MLGATE_SUPERGLUE_NATIVE=1: SuperPoint (threshold 0.005) +
    the GPU SuperGlue on a revisit pair of the synthetic sequence."""
    from mlgate import synthetic, verify
    monkeypatch.setenv("MLGATE_SUPERGLUE_NATIVE", "1")
    seq = synthetic.make_sequence(40, 8, 1)
    po = seq.place_of
    a, b = next((a, b) for a in range(40) for b in range(a + 1, 40) if po[a] == po[b])
    fr = synthetic.frames_host(seq, np.array([a, b]))
    m = verify.SuperGlue(device=str(dev))
    with pytest.warns(UserWarning, match="synthetic"):
        k0, k1, conf = m.detect_and_match(fr[0], fr[1])
    assert m._is_native
    assert k0.shape == k1.shape and k0.shape[1] == 2 and len(conf) == len(k0) and len(k0) > 20
    assert np.all(conf > 0.2)
    out = m.detect_and_match_batch(torch.from_numpy(fr).to(dev), [(0, 1)])
    assert np.array_equal(out[0][0], k0) and np.array_equal(out[0][2], conf)
