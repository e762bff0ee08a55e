"""The LoFTR oracle (oracle/loftr.py) and the host-side LoFTR preparation (mlgate/loftr.py):
weight key set, BatchNorm folding / conv packing against torch, the position encoding
against the oracle's torch formula, and the oracle's behaviour on the synthetic
sequence (a revisit gives many confident coarse matches, an unrelated pair few).
kornia is absent: the oracle's semantics are restated from its published default
configuration (parity unpinned)."""
import numpy as np
import torch
import torch.nn.functional as F

from mlgate import loftr as mlf
from mlgate import synthetic
from mlgate.weights import loftr_keys, loftr_state_dict
from oracle import loftr as ol


def test_state_dict_keys_and_shapes():
    sd = loftr_state_dict(0)
    assert sorted(sd) == sorted(loftr_keys())
    assert sd["backbone.layer2.0.conv1.weight"].shape == (196, 128, 3, 3)
    assert sd["loftr_coarse.layers.7.mlp.0.weight"].shape == (512, 512)
    assert sd["loftr_fine.layers.1.q_proj.weight"].shape == (128, 128)


def test_fold_and_pack_equal_torch_conv():
    sd = loftr_state_dict(0)
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.standard_normal((1, 196, 6, 5), dtype=np.float32))
    name, bn = "backbone.layer2.1.conv1", "backbone.layer2.1.bn1"
    t = {k: torch.from_numpy(v) for k, v in sd.items()}
    ref = F.batch_norm(F.conv2d(x, t[name + ".weight"], padding=1), t[bn + ".running_mean"], t[bn + ".running_var"],
                       t[bn + ".weight"], t[bn + ".bias"], False, 0.0, 1e-5)
    w, b = mlf.fold_bn(sd[name + ".weight"], sd, bn)
    P = mlf.pack_conv(w, 256, 256)  # [256, 9 * 256], column tap * 256 + c
    xp = F.pad(x, (1, 1, 1, 1))
    cols = torch.stack([xp[0, :, ky:ky + 6, kx:kx + 5] for ky in range(3) for kx in range(3)])  # [9, 196, 6, 5]
    colp = torch.zeros(9, 256, 6, 5)
    colp[:, :196] = cols
    got = torch.from_numpy(P) @ colp.reshape(9 * 256, -1) + torch.from_numpy(np.pad(b, (0, 60)))[:, None]
    assert torch.allclose(got[:196].reshape(196, 6, 5), ref[0], atol=1e-4, rtol=1e-4)
    assert torch.all(got[196:] == 0)


def test_position_encoding_matches_oracle():
    pe = mlf.position_encoding(60, 80)
    ref = ol.position_encoding(60, 80).reshape(256, -1).T.numpy()
    assert pe.shape == (4800, 256) and np.abs(pe - ref).max() < 1e-5


def test_oracle_matches_revisits_not_unrelated_frames():
    sd = loftr_state_dict(0)
    o = ol.Oracle(sd)
    seq = synthetic.make_sequence(40, 8, 1)
    po = seq.place_of
    a, b = next((a, b) for a in range(40) for b in range(a + 1, 40) if po[a] == po[b])
    c, d = next((a, b) for a in range(40) for b in range(a + 1, 40) if po[a] != po[b])
    fr = synthetic.frames_host(seq, np.array([a, b, c, d]))
    fr = fr[:, 120:360, 160:480]  # 240 x 320 crops keep the CPU time short
    k0, k1, conf = o.detect_and_match(fr[0], fr[1])
    u0, _, _ = o.detect_and_match(fr[2], fr[3])
    assert len(k0) >= 40 and len(u0) <= len(k0) // 5, (len(k0), len(u0))
    assert np.all(conf > 0.2) and np.all(k0 % 8 == 0)
