"""The SuperGlue oracle (oracle/superglue.py) and the host-side SuperGlue preparation
(mlgate/superglue.py): key set, the Sinkhorn marginal identities, BatchNorm folding +
head-major permutation + k-step packing against the oracle's raw-weight forward (the
exact GPU dataflow restated in float32), and the oracle's matching behaviour on
synthetic descriptor pairs.  magicleap's package and weights are absent: parity of the
oracle itself is unpinned (restated from the published model)."""
import numpy as np
import torch

from mlgate import superglue as msg
from mlgate.weights import superglue_keys, superglue_state_dict
from oracle import superglue as osg


def _unit(a):
    return (a / np.linalg.norm(a, axis=-1, keepdims=True)).astype(np.float32)


def synthetic_pair(seed, n_shared=200, n0=300, n1=280, noise=0.15, W=640, H=480):
    """Frame 0: n0 keypoints; frame 1: a shuffled noisy copy of n_shared of them plus
    fresh ones.  Returns (kp0, sc0, d0, kp1, sc1, d1, truth {i0: i1})."""
    rng = np.random.default_rng(seed)
    d0 = _unit(rng.standard_normal((n0, 256)))
    kp0 = (rng.random((n0, 2)) * [W, H]).astype(np.float32)
    sc0 = rng.uniform(0.005, 1.0, n0).astype(np.float32)
    src = rng.permutation(n0)[:n_shared]
    d1 = np.concatenate([_unit(d0[src] + noise * rng.standard_normal((n_shared, 256)) / 16),
                         _unit(rng.standard_normal((n1 - n_shared, 256)))])
    kp1 = np.concatenate([kp0[src] + rng.normal(0, 2, (n_shared, 2)), rng.random((n1 - n_shared, 2)) * [W, H]])
    sc1 = rng.uniform(0.005, 1.0, n1).astype(np.float32)
    order = rng.permutation(n1)
    inv = np.argsort(order)
    truth = {int(src[k]): int(inv[k]) for k in range(n_shared)}
    return kp0, sc0, d0, kp1[order].astype(np.float32), sc1[order], d1[order], truth


def test_state_dict_keys_and_shapes():
    sd = superglue_state_dict(0)
    assert sorted(sd) == sorted(superglue_keys())
    assert sd["kenc.encoder.0.weight"].shape == (32, 3, 1)
    assert sd["kenc.encoder.12.weight"].shape == (256, 256, 1)
    assert sd["gnn.layers.17.mlp.0.weight"].shape == (512, 512, 1)
    assert sd["gnn.layers.17.mlp.3.weight"].shape == (256, 512, 1)
    assert np.asarray(sd["bin_score"]).shape == ()


def test_sinkhorn_marginals():
    rng = np.random.default_rng(1)
    m, n = 37, 52
    S = torch.from_numpy(rng.standard_normal((m, n), dtype=np.float32) * 4)
    P = osg.log_optimal_transport(S, 1.0, 200)
    norm = -np.log(m + n)
    T = torch.exp(P.double() + norm)  # coupling
    mu = np.r_[np.full(m, 1 / (m + n)), n / (m + n)]
    nu = np.r_[np.full(n, 1 / (m + n)), m / (m + n)]
    assert np.allclose(T.sum(0).numpy(), nu, rtol=1e-4)  # exact after the last v update
    assert np.allclose(T.sum(1).numpy(), mu, rtol=1e-3)  # converged
    # zero iterations: Z - norm itself
    P0 = osg.log_optimal_transport(S, 1.0, 0)
    assert torch.allclose(P0[:m, :n], S - float(norm)) and abs(float(P0[m, n]) - (1.0 - norm)) < 1e-5


def _unpack_kstep(t):
    """[K/16, N, 16] -> [N, K]."""
    k16, n, _ = t.shape
    return t.permute(1, 0, 2).reshape(n, k16 * 16)


def test_packed_weights_reproduce_the_oracle():
    """Folded BN, head-major q / k / v rows + merge columns and k-step packing, run as
    the GPU runs them (one head = 64 contiguous columns), equal the raw-weight oracle."""
    sd = superglue_state_dict(0)
    w = msg.weight_list(sd, "cpu", gemm_dtype=torch.float32)
    kp0, sc0, d0, kp1, sc1, d1, _ = synthetic_pair(0, n_shared=40, n0=60, n1=50)
    W, H = 640, 480
    ref0, ref1 = osg.Oracle(sd).descriptors(kp0, sc0, d0, kp1, sc1, d1, W, H)

    def kenc(kp, sc):
        size = torch.tensor([W, H], dtype=torch.float32)
        x = torch.cat([(torch.from_numpy(kp) - size / 2) / (size.max() * 0.7), torch.from_numpy(sc)[:, None]], 1)
        for l in range(3):
            x = torch.relu(x @ w[l].T + w[3 + l])
        x = torch.relu(x @ w[6].T + w[7])
        return x @ w[8].T + w[9]

    def attend(q, k, v):
        o = []
        for h in range(4):
            s = q[:, 64 * h:64 * h + 64] @ k[:, 64 * h:64 * h + 64].T / 8
            o.append(torch.softmax(s, -1) @ v[:, 64 * h:64 * h + 64])
        return torch.cat(o, 1)

    def layer(i, x, src):
        Wqkv, bqkv, Wout, bout, Wf1, bf1, Wf2, bf2 = w[10 + 8 * i:18 + 8 * i]
        Wqkv = _unpack_kstep(Wqkv)
        q = x @ Wqkv[:256].T + bqkv[:256]
        k = src @ Wqkv[256:512].T + bqkv[256:512]
        v = src @ Wqkv[512:].T + bqkv[512:]
        msg_ = attend(q, k, v) @ _unpack_kstep(Wout).T + bout
        h = torch.relu(torch.cat([x, msg_], 1) @ _unpack_kstep(Wf1).T + bf1)
        return h @ _unpack_kstep(Wf2).T + bf2

    x0 = torch.from_numpy(d0) + kenc(kp0, sc0)
    x1 = torch.from_numpy(d1) + kenc(kp1, sc1)
    for i in range(18):
        s0, s1 = (x1, x0) if i % 2 else (x0, x1)
        x0, x1 = x0 + layer(i, x0, s0), x1 + layer(i, x1, s1)
    Wf, bfin = w[-2], w[-1]
    got0, got1 = x0 @ Wf.T + bfin, x1 @ Wf.T + bfin
    for g, r in ((got0, ref0), (got1, ref1)):
        assert torch.allclose(g, r, atol=2e-3, rtol=1e-4), float((g - r).abs().max())


def test_oracle_recovers_shared_points():
    sd = superglue_state_dict(0)
    kp0, sc0, d0, kp1, sc1, d1, truth = synthetic_pair(3)
    m, s = osg.Oracle(sd).match(kp0, sc0, d0, kp1, sc1, d1, 640, 480)
    assert len(m) >= 0.9 * len(truth)
    correct = sum(truth.get(int(i)) == int(j) for i, j in m)
    assert correct >= 0.97 * len(m)
    assert np.all(s > 0.2) and np.all(s <= 1.0 + 1e-6)
    assert np.all(np.diff(m[:, 0]) > 0) and len(set(m[:, 1].tolist())) == len(m)  # row order, one-to-one


def test_oracle_empty_side_and_bf16_emulation():
    sd = superglue_state_dict(0)
    kp0, sc0, d0, kp1, sc1, d1, truth = synthetic_pair(4, n_shared=60, n0=90, n1=80)
    m, s = osg.Oracle(sd).match(kp0, sc0, d0, kp1[:0], sc1[:0], d1[:0], 640, 480)
    assert m.shape == (0, 2) and s.shape == (0,)
    a, _ = osg.Oracle(sd).match(kp0, sc0, d0, kp1, sc1, d1, 640, 480)
    b, _ = osg.Oracle(sd, emulate_bf16=True).match(kp0, sc0, d0, kp1, sc1, d1, 640, 480)
    sa, sb = {tuple(r) for r in a.tolist()}, {tuple(r) for r in b.tolist()}
    assert len(sa & sb) >= 0.95 * max(len(sa), 1)
