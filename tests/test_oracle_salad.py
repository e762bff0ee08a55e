"""SALAD oracle (serizba/salad aggregator restated, oracle/salad.py) and the host-side
weight packing of the GPU path (mlgate/salad.py).  Parity unpinned: the salad package
and checkpoints are absent (SALAD place_recognition.py:357-368 never runs its native
branch), so these are the restatement's own identities."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import salad as osalad
from mlgate import weights as W
from mlgate.salad import pack_aggregator


def test_state_dict_keys_and_shapes():
    sd = W.salad_state_dict(seed=3)
    assert sorted(sd) == sorted(W.salad_keys())
    for k, shp in W.salad_aggregator_shapes().items():
        assert np.asarray(sd["aggregator." + k]).shape == shp, k
    assert len([k for k in sd if k.startswith("backbone.model.")]) == len(W.hub_keys())


def test_sinkhorn_column_marginals_are_exact_after_v_update():
    # after the final v update every column of P = exp(log P - norm) sums to 1 (incl. dust bin)
    g = torch.Generator().manual_seed(0)
    S = torch.randn(2, 64, 529, generator=g) * 2
    P = torch.exp(osalad.get_matching_probs(S, torch.tensor(1.0), 3))
    assert P.shape == (2, 65, 529)
    torch.testing.assert_close(P.sum(1), torch.ones(2, 529), atol=1e-5, rtol=0)
    # rows approach a_i * (n + m) = 1 (clusters) and n - m (dust bin) as iterations grow
    P50 = torch.exp(osalad.get_matching_probs(S, torch.tensor(1.0), 50))
    torch.testing.assert_close(P50[:, :64].sum(2), torch.ones(2, 64), atol=1e-3, rtol=0)
    torch.testing.assert_close(P50[:, 64].sum(1), torch.full((2,), 529.0 - 64), atol=1e-1, rtol=0)


def test_log_otp_solver_matches_plain_sinkhorn():
    # log-domain updates == scaling iterations K / (K v) ... in the exp domain
    g = torch.Generator().manual_seed(1)
    M = torch.randn(1, 5, 7, generator=g, dtype=torch.float64)
    la = torch.log(torch.full((1, 5), 1 / 5.0, dtype=torch.float64))
    lb = torch.log(torch.full((1, 7), 1 / 7.0, dtype=torch.float64))
    lp = osalad.log_otp_solver(la, lb, M, num_iters=4)
    K = torch.exp(M[0])
    a, b = torch.exp(la[0]), torch.exp(lb[0])
    u, v = torch.ones(5, dtype=torch.float64), torch.ones(7, dtype=torch.float64)
    for _ in range(4):
        u = a / (K @ v)
        v = b / (K.t() @ u)
    torch.testing.assert_close(torch.exp(lp[0]), u[:, None] * K * v[None, :], rtol=1e-12, atol=0)


def test_aggregate_structure():
    sd = W.salad_state_dict(seed=5)
    g = torch.Generator().manual_seed(2)
    tokens = torch.randn(2, 530, 768, generator=g)
    d = osalad.aggregate(tokens, sd)
    assert d.shape == (2, osalad.DESC_DIM)
    torch.testing.assert_close(d.norm(dim=1), torch.ones(2), atol=1e-5, rtol=0)
    # each cluster block (stride 64 over l) has equal norm: every cluster is unit before the global norm
    agg = d[:, 256:].reshape(2, 128, 64)
    cn = agg.norm(dim=1)
    torch.testing.assert_close(cn, cn[:, :1].expand_as(cn), atol=1e-5, rtol=0)
    # the token part and the clusters share the global scale 1 / sqrt(1 + 64)
    torch.testing.assert_close(d[:, :256].norm(dim=1), torch.full((2,), 1 / math.sqrt(65)), atol=1e-5, rtol=0)


def test_packed_weights_reproduce_the_aggregator_layers():
    sd = W.salad_state_dict(seed=6)
    (w1, b1, w2, b2, wt1, bt1, wt2, bt2), dust = pack_aggregator(sd)
    assert dust == 1.0 and w1.shape == (1024, 768) and w2.shape == (256, 1024)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(50, 768, generator=g, dtype=torch.float64)
    h = F.relu(x @ w1.double().t() + b1.double())
    y = h @ w2.double().t() + b2.double()
    a = "aggregator."
    t = lambda k: torch.as_tensor(np.asarray(sd[a + k])).double()  # noqa: E731
    f = F.linear(F.relu(F.linear(x, t("cluster_features.0.weight").flatten(1), t("cluster_features.0.bias"))),
                 t("cluster_features.3.weight").flatten(1), t("cluster_features.3.bias"))
    p = F.linear(F.relu(F.linear(x, t("score.0.weight").flatten(1), t("score.0.bias"))),
                 t("score.3.weight").flatten(1), t("score.3.bias"))
    torch.testing.assert_close(y[:, :128], f, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(y[:, 128:192], p, rtol=1e-12, atol=1e-12)
    assert torch.all(y[:, 192:] == 0)
    torch.testing.assert_close(wt1, t("token_features.0.weight").float())


def test_preprocess_keeps_channel_order():
    img = np.zeros((40, 50, 3), np.uint8)
    img[..., 0] = 200  # blue in BGR stays channel 0
    x = osalad._vit.preprocess(img, osalad.IMAGE_SIZE, swap_rb=False)
    assert x.shape == (1, 3, 322, 322)
    assert float(x[0, 0].mean()) > float(x[0, 2].mean())


@pytest.mark.slow
def test_extract_descriptor_runs():
    sd = W.salad_state_dict(seed=0)
    rng = np.random.default_rng(0)
    d = osalad.extract_descriptor(rng.integers(0, 256, (120, 160, 3), dtype=np.uint8), sd)
    assert d.shape == (8448,) and abs(np.linalg.norm(d) - 1) < 1e-5
