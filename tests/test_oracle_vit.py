"""Pin the oracle's ViT-B/14 restatement architecturally against an independent
implementation of the same network: transformers.Dinov2Model with the same seeded
weights at 518x518, where the hub pos-embed interpolation is the identity (CPU)."""
import numpy as np
import pytest
import torch

from mlgate.weights import synthetic_state_dict
from oracle import vit as ovit


def hf_model(sd):
    from transformers import Dinov2Config, Dinov2Model
    cfg = Dinov2Config(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072,
                       patch_size=14, image_size=518, layer_norm_eps=1e-6, hidden_act="gelu", qkv_bias=True,
                       layerscale_value=1.0)
    m = Dinov2Model(cfg).eval()
    t = {k: torch.from_numpy(v) for k, v in sd.items()}
    hf = {
        "embeddings.cls_token": t["cls_token"],
        "embeddings.position_embeddings": t["pos_embed"],
        "embeddings.patch_embeddings.projection.weight": t["patch_embed.proj.weight"],
        "embeddings.patch_embeddings.projection.bias": t["patch_embed.proj.bias"],
        "embeddings.mask_token": torch.zeros(1, 768),
        "layernorm.weight": t["norm.weight"],
        "layernorm.bias": t["norm.bias"],
    }
    for i in range(12):
        p, q = f"blocks.{i}.", f"encoder.layer.{i}."
        w, b = t[p + "attn.qkv.weight"], t[p + "attn.qkv.bias"]
        for j, nm in enumerate(("query", "key", "value")):
            hf[q + f"attention.attention.{nm}.weight"] = w[j * 768:(j + 1) * 768]
            hf[q + f"attention.attention.{nm}.bias"] = b[j * 768:(j + 1) * 768]
        hf[q + "attention.output.dense.weight"] = t[p + "attn.proj.weight"]
        hf[q + "attention.output.dense.bias"] = t[p + "attn.proj.bias"]
        hf[q + "layer_scale1.lambda1"] = t[p + "ls1.gamma"]
        hf[q + "layer_scale2.lambda1"] = t[p + "ls2.gamma"]
        for nm in ("norm1", "norm2"):
            hf[q + f"{nm}.weight"] = t[p + f"{nm}.weight"]
            hf[q + f"{nm}.bias"] = t[p + f"{nm}.bias"]
        for nm in ("fc1", "fc2"):
            hf[q + f"mlp.{nm}.weight"] = t[p + f"mlp.{nm}.weight"]
            hf[q + f"mlp.{nm}.bias"] = t[p + f"mlp.{nm}.bias"]
    missing, unexpected = m.load_state_dict(hf, strict=False)
    assert not unexpected and not [k for k in missing if "mask_token" not in k], (missing, unexpected)
    return m


@pytest.mark.slow
def test_oracle_vit_matches_transformers_dinov2():
    torch.set_num_threads(8)
    sd = synthetic_state_dict(3)
    m = hf_model(sd)
    rng = np.random.default_rng(0)
    x = ovit.preprocess(rng.integers(0, 256, (480, 640, 3), dtype=np.uint8), 518)
    with torch.no_grad():
        ref = m(pixel_values=x).last_hidden_state[:, 1:]
    ours = ovit.forward_tokens(x, sd)
    assert ours.shape == ref.shape == (1, 1369, 768)
    assert torch.allclose(ours, ref, rtol=0, atol=2e-4), (ours - ref).abs().max()


def test_pos_embed_resample_shape_and_identity():
    sd = synthetic_state_dict(0)
    pe = torch.from_numpy(sd["pos_embed"])
    assert ovit.interpolate_pos_embed(pe, 37) is not None and torch.equal(ovit.interpolate_pos_embed(pe, 37), pe)
    assert ovit.interpolate_pos_embed(pe, 23).shape == (1, 530, 768)
