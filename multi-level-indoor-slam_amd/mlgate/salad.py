"""SALAD descriptor engine on the mlgate HIP kernels (the native branch of ``SALAD``).

Reference: ``SALAD._load_model`` / ``extract_descriptor`` / ``_preprocess``
(place_recognition.py:357-410).  The reference builds ``salad.SALAD(out_dim=8448)``
(serizba/salad: a DINOv2 ViT-B/14 backbone + the optimal-transport aggregator) when
that package imports, else falls back to MixVPR; the package is absent wherever the
reference runs, so ``mlgate.vpr.SALAD`` keeps the fallback by default and this engine is
opt-in (``MLGATE_SALAD_NATIVE=1``), like SuperGlue's native branch.

Per batch of frames: preprocessing (cv2 INTER_LINEAR to 322 x 322, no channel swap,
ImageNet normalisation), the ViT forward, the final LayerNorm over every token, the
aggregator's 1x1-conv MLPs as two MFMA GEMMs, then per frame one workgroup for the token
MLP, the 3-iteration log-domain Sinkhorn, the cluster aggregation and the
normalisations (csrc/salad.hip).  Output float32 [B, 8448].
"""
import numpy as np
import torch

from . import _native
from .vit import VitB14
from .weights import SALAD_CLUSTER_DIM, SALAD_CLUSTERS, resolve_salad_state_dict

IMAGE_SIZE = 322  # SALAD's evaluation size; the hub PatchEmbed needs multiples of 14
DESC_DIM = SALAD_CLUSTERS * SALAD_CLUSTER_DIM + 256


def pack_aggregator(sd):
    """serizba/salad aggregator tensors -> the mlg_salad_weights order (include/mlgate.h)."""
    a = "aggregator."
    g = lambda k: torch.as_tensor(np.asarray(sd[a + k], np.float32))  # noqa: E731
    c0, s0 = g("cluster_features.0.weight").reshape(512, -1), g("score.0.weight").reshape(512, -1)
    w1 = torch.cat([c0, s0], 0)
    b1 = torch.cat([g("cluster_features.0.bias"), g("score.0.bias")])
    w2 = torch.zeros(256, 1024)
    w2[:SALAD_CLUSTER_DIM, :512] = g("cluster_features.3.weight").reshape(SALAD_CLUSTER_DIM, 512)
    w2[128:128 + SALAD_CLUSTERS, 512:] = g("score.3.weight").reshape(SALAD_CLUSTERS, 512)
    b2 = torch.zeros(256)
    b2[:SALAD_CLUSTER_DIM] = g("cluster_features.3.bias")
    b2[128:128 + SALAD_CLUSTERS] = g("score.3.bias")
    dust = float(np.asarray(sd[a + "dust_bin"], np.float32).reshape(()))
    return [w1, b1, w2, b2, g("token_features.0.weight"), g("token_features.0.bias"),
            g("token_features.2.weight"), g("token_features.2.bias")], dust


class SaladGPU:
    """Packed device weights for batched SALAD descriptor extraction."""

    def __init__(self, state_dict=None, device="cuda", max_batch=64, pretrained_path=None):
        if state_dict is None:
            state_dict, self.weights_source = resolve_salad_state_dict(pretrained_path)
        else:
            self.weights_source = "given"
        backbone = {k[len("backbone.model."):]: v for k, v in state_dict.items() if k.startswith("backbone.model.")}
        self._vit = VitB14(backbone, device=device, image_size=IMAGE_SIZE, max_batch=max_batch, pool="gem",
                           swap_rb=False, precise=False)  # mlg_salad_forward runs the plain bf16 trunk
        self.device = self._vit.device
        self.max_batch = max_batch
        agg, self.dust_bin = pack_aggregator(state_dict)
        bf = {0, 2}
        self._agg = [t.to(self.device, torch.bfloat16 if i in bf else torch.float32).contiguous()
                     for i, t in enumerate(agg)]

    def forward(self, frames):
        """frames: uint8 [B, H, W, C] (or [B, H, W]) device tensor -> float32 [B, 8448]."""
        if frames.dim() == 3:
            frames = frames.unsqueeze(-1)
        if frames.dtype != torch.uint8 or frames.device.type != "cuda":
            raise TypeError("frames must be a uint8 tensor on the HIP device")
        return _native.ops().salad_forward(frames.contiguous(), self._vit._w, self._agg, self.dust_bin, IMAGE_SIZE,
                                           self.max_batch)
