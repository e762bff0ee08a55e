"""Oracle for the LoFTR matcher (test infrastructure only).

The reference's ``LoFTR.detect_and_match`` (scripts/semantic_gating/geometric_verification.py:
458-526) runs ``kornia.feature.LoFTR(pretrained='indoor')`` (:446-449) on grayscale
frames: cv2 BGR2GRAY (:486-494), resize down to multiples of 8 (:497-504), /255 (:507-508),
then rescales the keypoints back (:521-526).  kornia (unpinned; absent here, with its
'indoor' checkpoint) is restated in torch fp32 on the CPU from its published default
configuration -- parity unpinned:

  * backbone ResNetFPN_8_2: conv7x7/2 (1 -> 128) + BN + ReLU; layer1..3 of two
    BasicBlocks each (dims 128, 196, 256; strides 1, 2, 2; 1x1 conv + BN shortcut where
    the stride is 2); FPN: 1x1 lateral convs, bilinear x2 upsampling (align_corners=True),
    conv3x3 + BN + LeakyReLU + conv3x3 merges; outputs 1/8 (256 ch) and 1/2 (128 ch);
  * PositionEncodingSine(256) with the reference-era div term (temp_bug_fix False for
    'indoor': exp(arange(0, 128, 2) * floor(-ln(1e4) / 256 / 2)));
  * LocalFeatureTransformer, 8 layers self/cross alternating (d 256, 8 heads, linear
    attention elu + 1, eps 1e-6; q/k/v/merge without bias; norm1 on the merged message;
    MLP [x | msg] 512 -> 512 -> ReLU -> 256; norm2; residual); the cross step updates
    feat1 from the already updated feat0;
  * CoarseMatching dual_softmax: sim = (f0 / 16)(f1 / 16)^T / 0.1, conf = softmax over
    dim 1 * softmax over dim 2, conf > 0.2, border_rm 2 cells, mutual max, first j per i;
  * FinePreprocess (window 5, stride 4, padding 2 unfold of the 1/2 map; down_proj of the
    coarse feature, merge_feat of the concatenation), a 2-layer fine transformer (d 128),
    FineMatching: softmax(center . window / sqrt(128)) -> spatial expectation on the
    normalised [-1, 1] grid; kpts1 += coords * 2 * 2 (W // 2 times the 1/2 -> 1 scale).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

BLOCK_DIMS = (128, 196, 256)
D_C, D_F, NHEAD, WIN = 256, 128, 8, 5
THR, BORDER, TEMP = 0.2, 2, 0.1
LAYERS_C = ("self", "cross") * 4
LAYERS_F = ("self", "cross")


def _bn(x, sd, p, eps=1e-5):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        False, 0.0, eps)


def _block(x, sd, p, stride):
    y = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"], stride=stride, padding=1), sd, p + ".bn1"))
    y = _bn(F.conv2d(y, sd[p + ".conv2.weight"], padding=1), sd, p + ".bn2")
    if stride != 1:
        x = _bn(F.conv2d(x, sd[p + ".downsample.0.weight"], stride=stride), sd, p + ".downsample.1")
    return F.relu(x + y)


def backbone(sd, img):
    """img f32 [B, 1, H, W] in [0, 1] -> (coarse [B, 256, H/8, W/8], fine [B, 128, H/2, W/2])."""
    b = "backbone."
    x0 = F.relu(_bn(F.conv2d(img, sd[b + "conv1.weight"], stride=2, padding=3), sd, b + "bn1"))
    x1 = _block(_block(x0, sd, b + "layer1.0", 1), sd, b + "layer1.1", 1)
    x2 = _block(_block(x1, sd, b + "layer2.0", 2), sd, b + "layer2.1", 1)
    x3 = _block(_block(x2, sd, b + "layer3.0", 2), sd, b + "layer3.1", 1)
    x3_out = F.conv2d(x3, sd[b + "layer3_outconv.weight"])
    up = lambda t: F.interpolate(t, scale_factor=2.0, mode="bilinear", align_corners=True)  # noqa: E731
    x2_out = F.conv2d(x2, sd[b + "layer2_outconv.weight"]) + up(x3_out)
    x2_out = F.leaky_relu(_bn(F.conv2d(x2_out, sd[b + "layer2_outconv2.0.weight"], padding=1), sd,
                              b + "layer2_outconv2.1"))
    x2_out = F.conv2d(x2_out, sd[b + "layer2_outconv2.3.weight"], padding=1)
    x1_out = F.conv2d(x1, sd[b + "layer1_outconv.weight"]) + up(x2_out)
    x1_out = F.leaky_relu(_bn(F.conv2d(x1_out, sd[b + "layer1_outconv2.0.weight"], padding=1), sd,
                              b + "layer1_outconv2.1"))
    x1_out = F.conv2d(x1_out, sd[b + "layer1_outconv2.3.weight"], padding=1)
    return x3_out, x1_out


def position_encoding(h, w, d=D_C):
    """PositionEncodingSine(d, temp_bug_fix=False) restricted to [d, h, w] (float32)."""
    y = torch.ones(h, w).cumsum(0).float().unsqueeze(0)
    x = torch.ones(h, w).cumsum(1).float().unsqueeze(0)
    div = torch.exp(torch.arange(0, d // 2, 2).float() * (-math.log(10000.0) / d // 2))[:, None, None]
    pe = torch.zeros(d, h, w)
    pe[0::4] = torch.sin(x * div)
    pe[1::4] = torch.cos(x * div)
    pe[2::4] = torch.sin(y * div)
    pe[3::4] = torch.cos(y * div)
    return pe


def _linear_attention(q, k, v, eps=1e-6):
    """LinearAttention on [N, L, H, D] (elu + 1 feature map)."""
    Q, K = F.elu(q) + 1, F.elu(k) + 1
    L = v.size(1)
    v = v / L
    KV = torch.einsum("nshd,nshv->nhdv", K, v)
    Z = 1 / (torch.einsum("nlhd,nhd->nlh", Q, K.sum(dim=1)) + eps)
    return torch.einsum("nlhd,nhdv,nlh->nlhv", Q, KV, Z) * L


def encoder_layer(sd, p, x, src, d):
    n = x.size(0)
    hd = d // NHEAD
    q = (x @ sd[p + ".q_proj.weight"].T).view(n, -1, NHEAD, hd)
    k = (src @ sd[p + ".k_proj.weight"].T).view(n, -1, NHEAD, hd)
    v = (src @ sd[p + ".v_proj.weight"].T).view(n, -1, NHEAD, hd)
    msg = _linear_attention(q, k, v).reshape(n, -1, d)
    msg = msg @ sd[p + ".merge.weight"].T
    msg = F.layer_norm(msg, (d,), sd[p + ".norm1.weight"], sd[p + ".norm1.bias"])
    msg = torch.cat([x, msg], dim=2)
    msg = F.relu(msg @ sd[p + ".mlp.0.weight"].T) @ sd[p + ".mlp.2.weight"].T
    msg = F.layer_norm(msg, (d,), sd[p + ".norm2.weight"], sd[p + ".norm2.bias"])
    return x + msg


def transformer(sd, prefix, f0, f1, names, d):
    for i, name in enumerate(names):
        p = f"{prefix}.layers.{i}"
        if name == "self":
            f0, f1 = encoder_layer(sd, p, f0, f0, d), encoder_layer(sd, p, f1, f1, d)
        else:
            f0 = encoder_layer(sd, p, f0, f1, d)
            f1 = encoder_layer(sd, p, f1, f0, d)
    return f0, f1


def coarse_matching(f0, f1, hc, wc):
    """[1, L, 256] x2 -> (i_ids, j_ids, mconf, conf)."""
    f0, f1 = f0 / f0.shape[-1] ** 0.5, f1 / f1.shape[-1] ** 0.5
    sim = torch.einsum("nlc,nsc->nls", f0, f1) / TEMP
    conf = F.softmax(sim, 1) * F.softmax(sim, 2)
    mask = (conf > THR).view(1, hc, wc, hc, wc)
    b = BORDER
    mask[:, :b] = False
    mask[:, :, :b] = False
    mask[:, :, :, :b] = False
    mask[:, :, :, :, :b] = False
    mask[:, -b:] = False
    mask[:, :, -b:] = False
    mask[:, :, :, -b:] = False
    mask[:, :, :, :, -b:] = False
    mask = mask.view(1, hc * wc, hc * wc)
    mask = mask & (conf == conf.max(dim=2, keepdim=True)[0]) & (conf == conf.max(dim=1, keepdim=True)[0])
    mask_v, all_j = mask.max(dim=2)
    b_ids, i_ids = torch.where(mask_v)
    j_ids = all_j[b_ids, i_ids]
    return i_ids, j_ids, conf[b_ids, i_ids, j_ids], conf


def fine_preprocess(sd, feat_f0, feat_f1, feat_c0, feat_c1, i_ids, j_ids, stride):
    W = WIN
    u0 = F.unfold(feat_f0, kernel_size=(W, W), stride=stride, padding=W // 2)
    u0 = u0.view(1, -1, W * W, u0.shape[-1]).permute(0, 3, 2, 1)  # n (c ww) l -> n l ww c
    u1 = F.unfold(feat_f1, kernel_size=(W, W), stride=stride, padding=W // 2)
    u1 = u1.view(1, -1, W * W, u1.shape[-1]).permute(0, 3, 2, 1)
    u0, u1 = u0[0, i_ids], u1[0, j_ids]
    c = torch.cat([feat_c0[0, i_ids], feat_c1[0, j_ids]], 0) @ sd["fine_preprocess.down_proj.weight"].T + \
        sd["fine_preprocess.down_proj.bias"]
    cat = torch.cat([torch.cat([u0, u1], 0), c[:, None, :].expand(-1, W * W, -1)], -1)
    m = cat @ sd["fine_preprocess.merge_feat.weight"].T + sd["fine_preprocess.merge_feat.bias"]
    return torch.chunk(m, 2, dim=0)


def fine_matching(f0, f1):
    """[M, 25, 128] x2 -> normalised expectation coords [M, 2] (x, y)."""
    M, WW, C = f0.shape
    W = int(math.sqrt(WW))
    sim = torch.einsum("mc,mrc->mr", f0[:, WW // 2, :], f1)
    heat = torch.softmax((1.0 / C ** 0.5) * sim, dim=1).view(-1, W, W)
    g = torch.linspace(-1.0, 1.0, W)
    gx = g[None, None, :].expand(1, W, W)
    gy = g[None, :, None].expand(1, W, W)
    return torch.stack([(heat * gx).sum((1, 2)), (heat * gy).sum((1, 2))], -1)


def to_gray(img_bgr):
    """cv2.cvtColor(BGR2GRAY) on uint8 (fixed point: (B 1868 + G 9617 + R 4899 + 2^13) >> 14)."""
    im = np.asarray(img_bgr)
    if im.ndim == 2:
        return im
    b, g, r = (im[..., c].astype(np.int32) for c in range(3))
    return ((b * 1868 + g * 9617 + r * 4899 + 8192) >> 14).astype(np.uint8)


class Oracle:
    def __init__(self, sd):
        self.sd = {k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in sd.items()}

    @torch.no_grad()
    def features(self, gray_u8):
        """uint8 [H, W] (H, W multiples of 8) -> coarse [1, 256, H/8, W/8], fine [1, 128, H/2, W/2]."""
        img = torch.from_numpy(np.asarray(gray_u8, np.uint8)).float()[None, None] / 255.0
        return backbone(self.sd, img)

    @torch.no_grad()
    def match_features(self, c0, f0, c1, f1, H):
        """LoFTR.forward after the backbone: -> dict(kpts0, kpts1, conf, i_ids, j_ids, conf_matrix)."""
        hc, wc = c0.shape[2:]
        pe = position_encoding(hc, wc)
        t0 = (c0 + pe[None]).flatten(2).transpose(1, 2)
        t1 = (c1 + pe[None]).flatten(2).transpose(1, 2)
        t0, t1 = transformer(self.sd, "loftr_coarse", t0, t1, LAYERS_C, D_C)
        i_ids, j_ids, mconf, conf = coarse_matching(t0, t1, hc, wc)
        scale_c = H / hc
        k0 = torch.stack([i_ids % wc, i_ids // wc], 1) * scale_c
        k1 = torch.stack([j_ids % wc, j_ids // wc], 1) * scale_c
        out = {"i_ids": i_ids, "j_ids": j_ids, "conf": mconf, "conf_matrix": conf[0], "coarse0": t0[0],
               "coarse1": t1[0]}
        if len(i_ids) == 0:
            out.update(kpts0=k0.float(), kpts1=k1.float())
            return out
        stride = f0.shape[2] // hc
        w0, w1 = fine_preprocess(self.sd, f0, f1, t0, t1, i_ids, j_ids, stride)
        w0, w1 = transformer(self.sd, "loftr_fine", w0, w1, LAYERS_F, D_F)
        coords = fine_matching(w0, w1)
        scale_f = H / f0.shape[2]
        out.update(kpts0=k0.float(), kpts1=(k1 + coords * (WIN // 2) * scale_f).float(), expec=coords)
        return out

    def detect_and_match(self, img0, img1):
        """geometric_verification.py:484-526 with the restated model: gray, cv2.resize
        INTER_LINEAR down to multiples of 8 (oracle/csrc/oracle.c restatement; a same-size
        resize is cv2's copy), match, keypoints scaled back (float64, as :521-526)."""
        from . import _lib
        g0, g1 = to_gray(img0), to_gray(img1)
        if g0.shape != g1.shape:
            raise ValueError("oracle: frames must share a shape")
        h, w = g0.shape
        nh, nw = h // 8 * 8, w // 8 * 8
        if (nh, nw) != (h, w):
            g0, g1 = (_lib.resize_linear_u8(g[..., None], nh, nw)[..., 0] for g in (g0, g1))
        c0, f0 = self.features(g0)
        c1, f1 = self.features(g1)
        r = self.match_features(c0, f0, c1, f1, nh)
        sc = np.array([w / nw, h / nh])
        return r["kpts0"].numpy() * sc, r["kpts1"].numpy() * sc, r["conf"].numpy()
