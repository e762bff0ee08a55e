"""ResNet-50 fallback descriptor (MixVPR / SALAD) on the GPU vs the oracle
(oracle/resnet.py, whose resize is pinned bit-exact to Pillow and whose network is
pinned to transformers.ResNetModel).  The resize is bit-exact; descriptors (bf16 MFMA
GEMMs, f32 residual stream, BN folded) within 1 - cos <= 2e-3 of the fp32 oracle."""
import numpy as np
import pytest
import torch

from mlgate import _native
from mlgate.resnet import ResNet50GPU
from mlgate.vpr import MixVPR, SALAD
from mlgate.weights import resnet50_state_dict
from oracle import resnet as ors

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,c", [((480, 640), 3), ((540, 720), 3), ((100, 90), 1), ((300, 200), 4)])
def test_pillow_resize_bit_exact(dev, shape, c):
    rng = np.random.default_rng(shape[0])
    imgs = rng.integers(0, 256, (2,) + shape + (c,), dtype=np.uint8)
    t = torch.from_numpy(imgs).to(dev)
    L = _native.lib()
    nb = L.mlg_resnet50_workspace_bytes(2, shape[0], shape[1])
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    out = torch.empty(2, 224, 224, 3, dtype=torch.uint8, device=dev)
    _native.check(L.mlg_op_pillow_resize_224(_native.ptr(t), 2, shape[0], shape[1], c, shape[0] * shape[1] * c,
                                             _native.ptr(ws), nb, _native.ptr(out), _native.stream_of(dev)), "resize")
    for b in range(2):
        img = imgs[b]
        img = np.repeat(img, 3, axis=2) if c == 1 else img[..., :3]
        assert np.array_equal(out[b].cpu().numpy(), ors.pil_resize_bilinear(img, (224, 224)))


def test_resnet_descriptor_matches_oracle(dev):
    sd = resnet50_state_dict(0)
    rng = np.random.default_rng(1)
    imgs = rng.integers(0, 256, (3, 480, 640, 3), dtype=np.uint8)
    net = ResNet50GPU(sd, device=str(dev))
    got = net.forward_device(torch.from_numpy(imgs).to(dev), 4096).cpu().numpy()
    for b in range(3):
        ref = ors.extract_descriptor(sd, imgs[b], 4096)
        assert np.all(got[b, 2048:] == 0)
        cos = float(np.dot(got[b], ref) / (np.linalg.norm(got[b]) * np.linalg.norm(ref)))
        assert 1 - cos <= 2e-3, 1 - cos
        assert np.linalg.norm(got[b] - ref) / np.linalg.norm(ref) < 0.05


def test_mixvpr_salad_dropin(dev):
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)
    with pytest.warns(UserWarning):
        m = MixVPR(device=str(dev))
        d = m.extract_descriptor(img)
    assert d.shape == (4096,) and d.dtype == np.float32
    s = SALAD(device=str(dev))
    ds = s.extract_descriptor(img)
    assert ds.shape == (8448,) and np.allclose(ds[:2048], d[:2048]) and np.all(ds[2048:] == 0)
    gray = img[..., 0]
    assert m.extract_descriptor(gray).shape == (4096,)
