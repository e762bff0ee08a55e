"""The ResNet-50 fallback oracle (oracle/resnet.py): Pillow resize restatement pinned
bit-exact against Pillow itself; the network restatement pinned against
transformers.ResNetModel (same architecture, torchvision v1.5 stride placement) with
the same seeded weights."""
import numpy as np
import pytest
import torch

from mlgate.weights import resnet50_state_dict
from oracle import resnet as ors


@pytest.mark.parametrize("shape", [(480, 640), (540, 720), (100, 90), (224, 300), (37, 500), (224, 224)])
def test_pil_resize_restatement_bit_exact(shape):
    from PIL import Image
    rng = np.random.default_rng(sum(shape))
    img = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(img).resize((224, 224), Image.BILINEAR))
    assert np.array_equal(ors.pil_resize_bilinear(img, (224, 224)), ref)


def _hf_model(sd):
    from transformers import ResNetConfig, ResNetModel
    cfg = ResNetConfig(num_channels=3, embedding_size=64, hidden_sizes=[256, 512, 1024, 2048], depths=[3, 4, 6, 3],
                       layer_type="bottleneck", hidden_act="relu", downsample_in_first_stage=False,
                       downsample_in_bottleneck=False)
    m = ResNetModel(cfg).eval()
    hf = {}
    bn = ("weight", "bias", "running_mean", "running_var")
    hf["embedder.embedder.convolution.weight"] = sd["conv1.weight"]
    for s in bn:
        hf[f"embedder.embedder.normalization.{s}"] = sd[f"bn1.{s}"]
    for li, (_, blocks, _) in enumerate(ors.STAGES):
        for b in range(blocks):
            p, q = f"layer{li + 1}.{b}.", f"encoder.stages.{li}.layers.{b}."
            for c in range(3):
                hf[q + f"layer.{c}.convolution.weight"] = sd[p + f"conv{c + 1}.weight"]
                for s in bn:
                    hf[q + f"layer.{c}.normalization.{s}"] = sd[p + f"bn{c + 1}.{s}"]
            if b == 0:
                hf[q + "shortcut.convolution.weight"] = sd[p + "downsample.0.weight"]
                for s in bn:
                    hf[q + f"shortcut.normalization.{s}"] = sd[p + f"downsample.1.{s}"]
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in hf.items()},
                                            strict=False)
    assert not unexpected and all("num_batches_tracked" in k for k in missing), (missing, unexpected)
    return m


def test_resnet_restatement_matches_transformers():
    sd = resnet50_state_dict(0)
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)
    x = ors.preprocess(img)[None]
    with torch.no_grad():
        ref = _hf_model(sd)(pixel_values=x).pooler_output.flatten()
        got = ors.resnet50_features(sd, x).flatten()
    assert torch.allclose(got, ref, rtol=1e-4, atol=1e-5), (got - ref).abs().max()
    d = ors.extract_descriptor(sd, img, 4096)
    assert d.shape == (4096,) and np.all(d[2048:] == 0)
    assert ors.extract_descriptor(sd, img, 1000).shape == (1000,)
