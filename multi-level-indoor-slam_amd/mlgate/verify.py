"""Geometric verification: drop-in mirror of scripts/semantic_gating/geometric_verification.py.

The dataclasses, the verifier decision rule (geometric_verification.py:586-634),
the semantic cross-floor skip and its statistics (:688-744), SuperPoint + LightGlue
matching (:196-312; mlgate.superpoint / mlgate.lightglue), detector-free LoFTR
(:424-526; mlgate.loftr) and the RANSAC stage -- essential / fundamental matrix +
recoverPose (:104-188; mlgate.geometry) -- all run on the GPU.  SuperGlue resolves to
the LightGlue path exactly as the reference does (its native branch defers to it), or,
opted in, to the GPU SuperGlue + Sinkhorn matcher the class configures (mlgate.superglue).
"""
import os
import warnings
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import geometry


@dataclass
class MatchResult:
    """Outcome of verifying one (query, match) keyframe pair."""
    query_idx: int
    match_idx: int
    num_keypoints_query: int
    num_keypoints_match: int
    num_matches: int
    num_inliers: int
    inlier_ratio: float
    relative_pose: Optional[np.ndarray]
    essential_matrix: Optional[np.ndarray]
    confidence: float
    is_valid: bool


@dataclass
class Keypoint:
    x: float
    y: float
    score: float
    descriptor: Optional[np.ndarray] = None


def _rejected(query_idx, match_idx):
    return MatchResult(query_idx=query_idx, match_idx=match_idx, num_keypoints_query=0, num_keypoints_match=0,
                       num_matches=0, num_inliers=0, inlier_ratio=0.0, relative_pose=None, essential_matrix=None,
                       confidence=0.0, is_valid=False)


class BaseFeatureMatcher:
    def __init__(self, device: str = 'cuda'):
        self.device = device
        self.model = None
        self.ransac_hypotheses = geometry.DEFAULT_HYPOTHESES
        self.ransac_seed = 0

    def detect_and_match(self, image1: np.ndarray, image2: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        raise NotImplementedError

    def verify_geometric_consistency(self, kpts1: np.ndarray, kpts2: np.ndarray, K: Optional[np.ndarray] = None,
                                     ransac_threshold: float = 3.0) -> Tuple[np.ndarray, np.ndarray, float]:
        """cv2.findEssentialMat (K given) / cv2.findFundamentalMat (FM_RANSAC) on the GPU."""
        if len(kpts1) < 5:
            return np.array([]), None, 0.0
        r = geometry.epipolar_ransac([kpts1], [kpts2], K, ransac_threshold, self.ransac_hypotheses,
                                     self.ransac_seed, self.device, with_pose=False)[0]
        if r.model is None:
            return np.array([]), None, 0.0
        return r.mask, r.model, float(np.sum(r.mask) / len(kpts1))

    def estimate_relative_pose(self, kpts1: np.ndarray, kpts2: np.ndarray, K: np.ndarray, inlier_mask: np.ndarray,
                               E: np.ndarray) -> Optional[np.ndarray]:
        """cv2.recoverPose(E, kpts1[mask], kpts2[mask], K) on the GPU -> 4x4 [R|t]."""
        if E is None or np.sum(inlier_mask) < 5:
            return None
        return geometry.recover_pose(kpts1, kpts2, K, inlier_mask, E, self.device)


class LightGlue(BaseFeatureMatcher):
    """SuperPoint + LightGlue on the GPU (geometric_verification.py:196-312).

    ``detect_and_match`` runs SuperPoint on both images (mlg_superpoint) and LightGlue
    on the pair (mlg_lightglue); ``detect_and_match_batch`` does the same for many
    pairs of device-resident keyframes with one SuperPoint launch sequence over the
    distinct frames and one LightGlue call over all pairs.  Weights: checkpoints from
    MLGATE_SUPERPOINT_WEIGHTS / MLGATE_LIGHTGLUE_WEIGHTS, else seeded synthetic ones
    (there is no network for the package's downloads).
    """

    def __init__(self, device: str = 'cuda', max_keypoints: int = 2048, detection_threshold: float = 0.001):
        super().__init__(device)
        self.max_keypoints = max_keypoints
        self.detection_threshold = detection_threshold
        self._model_loaded = False

    def _load_model(self):
        if self._model_loaded:
            return
        if os.environ.get("MLGATE_LIGHTGLUE_FALLBACK", "").lower() in ("1", "orb"):
            # the reference's ImportError branch (:237-242), selected explicitly: the
            # GPU SuperPoint + LightGlue are always available here
            warnings.warn("LightGlue not installed. Using ORB+BFMatcher fallback. "
                          "Install with: pip install git+https://github.com/cvg/LightGlue.git")
            self._load_fallback()
            return
        from .lightglue import LightGlueGPU
        from .superpoint import SuperPointGPU
        self.extractor = SuperPointGPU(device=self.device, max_num_keypoints=self.max_keypoints,
                                       detection_threshold=self.detection_threshold)
        self.matcher = LightGlueGPU(device=self.device)
        synth = [n for n, m in (("SuperPoint", self.extractor), ("LightGlue", self.matcher))
                 if m.weights_source.startswith("synthetic")]
        if synth:
            warnings.warn(f"{' and '.join(synth)} weights not configured (MLGATE_SUPERPOINT_WEIGHTS / "
                          "MLGATE_LIGHTGLUE_WEIGHTS); using seeded synthetic weights")
        self._model_loaded = True
        self._is_native = True

    def _load_fallback(self):
        """cv2.ORB_create(nfeatures=max_keypoints) + BFMatcher(NORM_HAMMING, crossCheck)
        (:244-248) as the GPU ORB (mlgate.orb, csrc/orb.hip)."""
        from .orb import OrbGPU
        self.orb = OrbGPU(device=self.device, nfeatures=self.max_keypoints)
        self.bf = self.orb
        self._model_loaded = True
        self._is_native = False

    def _detect_and_match_fallback(self, image1: np.ndarray, image2: np.ndarray):
        """:314-350 -- ORB on both frames, cross-checked Hamming matches sorted by distance,
        confidence 1 - distance / max distance."""
        return self._fallback_pairs([image1, image2], [(0, 1)])[0]

    def _fallback_pairs(self, images, pairs):
        if not hasattr(self, "orb"):
            self._load_fallback()
        frames = [np.asarray(im) for im in images]
        groups = {}
        for i, f in enumerate(frames):
            groups.setdefault(f.shape, []).append(i)
        feats = {}
        for shape, idx in groups.items():  # one launch sequence per frame size
            batch = torch.from_numpy(np.ascontiguousarray(np.stack([frames[i] for i in idx]))).to(self.orb.device)
            if batch.dim() == 3:
                batch = batch.unsqueeze(-1)
            kp, _, _, _, ds, cnt = self.orb.detect_device(batch)
            for j, i in enumerate(idx):
                feats[i] = (kp[j], ds[j], cnt[j])
        return self._match_feats(feats, pairs)

    def _match_feats(self, feats, pairs):
        out = []
        for a, b in pairs:
            ka, da, na = feats[a]
            kb, db, nb = feats[b]
            n1, n2 = int(na), int(nb)
            if n1 == 0 or n2 == 0 or n1 < 5 or n2 < 5:
                out.append((np.array([]), np.array([]), np.array([])))
                continue
            desc = torch.stack([da, db])
            cnt = torch.tensor([n1, n2], dtype=torch.int32, device=desc.device)
            q, t, d, n = self.orb.match_device(desc, cnt, [0], [1])
            m = int(n[0])
            q, t, d = q[0, :m].cpu().numpy(), t[0, :m].cpu().numpy(), d[0, :m].cpu().numpy()
            k1, k2 = ka.cpu().numpy(), kb.cpu().numpy()
            m1 = np.array([k1[i].tolist() for i in q])
            m2 = np.array([k2[j].tolist() for j in t])
            max_dist = max(float(x) for x in d) if m else 1
            out.append((m1, m2, np.array([1 - float(x) / max_dist for x in d])))
        return out

    def detect_and_match(self, image1: np.ndarray, image2: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        self._load_model()
        if not getattr(self, "_is_native", False):
            return self._detect_and_match_fallback(image1, image2)
        if np.shape(image1) == np.shape(image2):
            f1, f2 = self.extractor.extract([image1, image2])
        else:
            f1, = self.extractor.extract([image1])
            f2, = self.extractor.extract([image2])
        m, sc, _ = self.matcher.match(f1, f2)
        return (f1["keypoints"][m[:, 0]].astype(np.float32), f2["keypoints"][m[:, 1]].astype(np.float32),
                sc.astype(np.float32))

    def detect_and_match_batch(self, frames, pairs):
        """frames: device uint8 [F, H, W, C]; pairs: [(a, b), ...] frame indices ->
        list of (kpts_a [S, 2], kpts_b [S, 2], scores [S]) numpy arrays per pair."""
        self._load_model()
        pairs = list(pairs)
        if not pairs:
            return []
        if not getattr(self, "_is_native", False):  # ORB fallback: one detect over the used frames
            used = sorted({i for p in pairs for i in p})
            sel = frames[torch.as_tensor(used, device=frames.device)]
            kp, _, _, _, ds, cnt = self.orb.detect_device(sel)
            feats = {f: (kp[j], ds[j], cnt[j]) for j, f in enumerate(used)}
            return self._match_feats(feats, pairs)
        used = sorted({i for p in pairs for i in p})
        pos = {f: j for j, f in enumerate(used)}
        sel = frames[torch.as_tensor(used, device=frames.device)] if len(used) < frames.shape[0] else frames
        kp, _, ds, _, cnt = self.extractor.extract_device(sel)
        counts = cnt.cpu().numpy()
        m, sc, n, _ = self.matcher.match_device(kp, ds, counts, [pos[a] for a, _ in pairs],
                                                [pos[b] for _, b in pairs])
        kp, m, sc, n = kp.cpu().numpy(), m.cpu().numpy(), sc.cpu().numpy(), n.cpu().numpy()
        out = []
        for p, (a, b) in enumerate(pairs):
            mm = m[p, :n[p]]
            out.append((kp[pos[a]][mm[:, 0]], kp[pos[b]][mm[:, 1]], sc[p, :n[p]]))
        return out


class SuperGlue(BaseFeatureMatcher):
    """geometric_verification.py:353-421.  The reference's native branch never runs
    SuperGlue (:419-421 return the LightGlue fallback, and the magicleap package is
    absent), so by default this matcher IS the GPU LightGlue path, with the reference's
    warning.  ``MLGATE_SUPERGLUE_NATIVE=1`` (or ``.native = True``) selects the model the
    class configures instead: magicleap SuperPoint settings (nms_radius 4,
    keypoint_threshold 0.005, max_keypoints) + SuperGlue (sinkhorn_iterations 20,
    match_threshold 0.2) on the GPU (mlgate.superglue, csrc/superglue.hip); weights from
    MLGATE_SUPERGLUE_WEIGHTS, else seeded synthetic ones."""

    def __init__(self, device: str = 'cuda', max_keypoints: int = 2048, weights: str = 'indoor'):
        super().__init__(device)
        self.max_keypoints = max_keypoints
        self.weights = weights
        self.native = None  # None: MLGATE_SUPERGLUE_NATIVE decides; True / False force it
        self._model_loaded = False

    def _load_model(self):
        if self._model_loaded:
            return
        native = self.native if self.native is not None else os.environ.get("MLGATE_SUPERGLUE_NATIVE") == "1"
        if native:
            from .superglue import SuperGlueGPU
            from .superpoint import SuperPointGPU
            self.extractor = SuperPointGPU(device=self.device, max_num_keypoints=self.max_keypoints,
                                           detection_threshold=0.005, nms_radius=4)
            self.matcher = SuperGlueGPU(device=self.device)
            synth = [n for n, m in (("SuperPoint", self.extractor), ("SuperGlue", self.matcher))
                     if m.weights_source.startswith("synthetic")]
            if synth:
                warnings.warn(f"{' and '.join(synth)} weights not configured (MLGATE_SUPERPOINT_WEIGHTS / "
                              "MLGATE_SUPERGLUE_WEIGHTS); using seeded synthetic weights")
            self._is_native = True
        else:
            warnings.warn("SuperGlue not installed. Using LightGlue fallback.")
            self._fallback = LightGlue(device=self.device, max_keypoints=self.max_keypoints)
            self._is_native = False
        self._model_loaded = True

    def detect_and_match(self, image1, image2):
        self._load_model()
        if not self._is_native:
            return self._fallback.detect_and_match(image1, image2)
        if np.shape(image1) != np.shape(image2):
            raise ValueError("SuperGlue: the two frames must share a shape (one normalisation size per batch)")
        h, w = np.shape(image1)[:2]
        f1, f2 = self.extractor.extract([image1, image2])
        m, sc = self.matcher.match(f1, f2, w, h)
        return (f1["keypoints"][m[:, 0]].astype(np.float32), f2["keypoints"][m[:, 1]].astype(np.float32),
                sc.astype(np.float32))

    def detect_and_match_batch(self, frames, pairs):
        """frames: device uint8 [F, H, W, C]; pairs: [(a, b), ...] -> list of
        (kpts_a [S, 2], kpts_b [S, 2], scores [S]) numpy arrays per pair."""
        self._load_model()
        if not self._is_native:
            return self._fallback.detect_and_match_batch(frames, pairs)
        pairs = list(pairs)
        if not pairs:
            return []
        used = sorted({i for p in pairs for i in p})
        pos = {f: j for j, f in enumerate(used)}
        sel = frames[torch.as_tensor(used, device=frames.device)] if len(used) < frames.shape[0] else frames
        kp, sc, ds, _, cnt = self.extractor.extract_device(sel)
        m, s, n = self.matcher.match_device(kp, sc, ds, cnt.cpu().numpy(), [pos[a] for a, _ in pairs],
                                            [pos[b] for _, b in pairs], int(frames.shape[2]), int(frames.shape[1]))
        kp, m, s, n = kp.cpu().numpy(), m.cpu().numpy(), s.cpu().numpy(), n.cpu().numpy()
        return [(kp[pos[a]][m[p, :n[p], 0]], kp[pos[b]][m[p, :n[p], 1]], s[p, :n[p]]) for p, (a, b) in enumerate(pairs)]


class LoFTR(BaseFeatureMatcher):
    """geometric_verification.py:424-526.  The reference runs kornia's LoFTR when kornia
    imports (pretrained `weights`) and otherwise warns and uses the LightGlue fallback
    (:447-467).  kornia and its checkpoints are absent here, so by default this class
    behaves like the reference in that environment: the warning, then the GPU LightGlue
    path.  The native detector-free matcher -- kornia.feature.LoFTR on cv2 BGR2GRAY frames
    resized down to multiples of 8 (cv2 INTER_LINEAR), /255, keypoints scaled back
    (mlgate.loftr, csrc/loftr.hip) -- is opt-in: ``MLGATE_LOFTR_NATIVE=1``, a checkpoint in
    ``MLGATE_LOFTR_WEIGHTS``, or ``.native = True``.  It is the 'indoor' configuration;
    'outdoor' needs its checkpoint in MLGATE_LOFTR_WEIGHTS (otherwise the fallback is
    used).  The native kernels match frames of one shape; a pair of differently shaped
    frames is matched by the LightGlue fallback, with a warning."""

    def __init__(self, device: str = 'cuda', weights: str = 'indoor'):
        super().__init__(device)
        self.weights = weights
        self.native = None  # None: the environment decides (see the class docstring)
        self._model_loaded = False

    def _want_native(self):
        if self.native is not None:
            return bool(self.native)
        return os.environ.get("MLGATE_LOFTR_NATIVE") == "1" or bool(os.environ.get("MLGATE_LOFTR_WEIGHTS"))

    def _load_model(self):
        if self._model_loaded:
            return
        native = self._want_native()
        if native and self.weights != 'indoor' and not os.environ.get("MLGATE_LOFTR_WEIGHTS"):
            warnings.warn(f"LoFTR weights {self.weights!r}: no checkpoint in MLGATE_LOFTR_WEIGHTS; "
                          "using the LightGlue fallback")
            native = False
        if native:
            from .loftr import LoFTRGPU
            self._matcher = LoFTRGPU(device=self.device)
            if self._matcher.weights_source.startswith("synthetic"):
                warnings.warn("LoFTR weights not configured (MLGATE_LOFTR_WEIGHTS); using seeded synthetic weights")
            self._is_native = True
        else:
            warnings.warn("LoFTR (kornia) not installed. Using LightGlue fallback. Install with: pip install kornia")
            self._fallback = LightGlue(device=self.device)
            self._is_native = False
        self._model_loaded = True

    @staticmethod
    def _scale(shape):
        h, w = shape[:2]
        return np.array([w / (w // 8 * 8), h / (h // 8 * 8)])  # float64, as :521-522

    def detect_and_match(self, image1: np.ndarray, image2: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        self._load_model()
        if not self._is_native:
            return self._fallback.detect_and_match(image1, image2)
        im1, im2 = np.asarray(image1, np.uint8), np.asarray(image2, np.uint8)
        if im1.shape != im2.shape:
            warnings.warn("LoFTR: frames of different shapes are matched by the LightGlue fallback")
            if not hasattr(self, "_fallback"):
                self._fallback = LightGlue(device=self.device)
            return self._fallback.detect_and_match(image1, image2)
        dev = torch.device(self.device)
        as4 = lambda im: torch.from_numpy(np.ascontiguousarray(im if im.ndim == 3 else im[..., None]))  # noqa: E731
        k0, k1, c = self._matcher.match_frames(torch.stack([as4(im1), as4(im2)]).to(dev), [(0, 1)])[0]
        sc = self._scale(im1.shape)
        return k0 * sc, k1 * sc, c

    def detect_and_match_batch(self, frames, pairs):
        """frames: device uint8 [F, H, W, C]; pairs [(a, b)] -> [(kpts_a, kpts_b, conf)]."""
        self._load_model()
        if not self._is_native:
            return self._fallback.detect_and_match_batch(frames, pairs)
        sc = self._scale(tuple(frames.shape[1:3]))
        return [(a * sc, b * sc, c) for a, b, c in self._matcher.match_frames(frames, pairs)]


_MATCHERS = {'lightglue': LightGlue, 'superglue': SuperGlue, 'loftr': LoFTR}


class GeometricVerifier:
    """Matching + RANSAC + the validity / confidence rule of the reference."""

    def __init__(self, matcher_type: str = 'lightglue', device: str = 'cuda', min_inliers: int = 20,
                 min_inlier_ratio: float = 0.25, ransac_threshold: float = 3.0):
        self.min_inliers = min_inliers
        self.min_inlier_ratio = min_inlier_ratio
        self.ransac_threshold = ransac_threshold
        cls = _MATCHERS.get(matcher_type.lower())
        if cls is None:
            raise ValueError(f"Unknown matcher: {matcher_type}")
        self.matcher = cls(device=device)

    def decide(self, kpts1, kpts2, inlier_mask, E, inlier_ratio, K=None, query_idx=0, match_idx=0) -> MatchResult:
        """The decision rule given matches and a RANSAC result (geometric_verification.py:606-634)."""
        n_in = int(np.sum(inlier_mask)) if len(inlier_mask) > 0 else 0
        pose = None
        if K is not None and E is not None and n_in >= 5:
            pose = self.matcher.estimate_relative_pose(kpts1, kpts2, K, inlier_mask, E)
        return MatchResult(query_idx=query_idx, match_idx=match_idx, num_keypoints_query=len(kpts1),
                           num_keypoints_match=len(kpts2), num_matches=len(kpts1), num_inliers=n_in,
                           inlier_ratio=inlier_ratio, relative_pose=pose, essential_matrix=E,
                           confidence=min(1.0, inlier_ratio * (n_in / self.min_inliers)),
                           is_valid=n_in >= self.min_inliers and inlier_ratio >= self.min_inlier_ratio)

    def verify(self, image1: np.ndarray, image2: np.ndarray, K: Optional[np.ndarray] = None, query_idx: int = 0,
               match_idx: int = 0) -> MatchResult:
        k1, k2, _ = self.matcher.detect_and_match(image1, image2)
        if len(k1) < 5:
            return _rejected(query_idx, match_idx)
        mask, E, ratio = self.matcher.verify_geometric_consistency(k1, k2, K, self.ransac_threshold)
        return self.decide(k1, k2, mask, E, ratio, K, query_idx, match_idx)

    def verify_matches_batch(self, matches: List[Tuple[np.ndarray, np.ndarray]], K: Optional[np.ndarray] = None,
                             indices: Optional[List[Tuple[int, int]]] = None) -> List[MatchResult]:
        """verify() for already-matched keypoints of many pairs: ONE batched GPU RANSAC +
        recoverPose over all pairs, then the reference's decision rule per pair."""
        run = [i for i, (k1, _) in enumerate(matches) if len(k1) >= 5]
        res = geometry.epipolar_ransac([matches[i][0] for i in run], [matches[i][1] for i in run], K,
                                       self.ransac_threshold, self.matcher.ransac_hypotheses,
                                       self.matcher.ransac_seed, self.matcher.device, with_pose=K is not None)
        by_pair = dict(zip(run, res))
        out = []
        for i, (k1, k2) in enumerate(matches):
            q, m = indices[i] if indices is not None else (i, i)
            r = by_pair.get(i)
            if r is None:
                out.append(_rejected(q, m))
                continue
            if r.model is None:
                mask, E, ratio = np.array([]), None, 0.0
            else:
                mask, E, ratio = r.mask, r.model, float(np.sum(r.mask) / len(k1))
            n_in = int(np.sum(mask)) if len(mask) > 0 else 0
            pose = r.pose if (K is not None and E is not None and n_in >= 5) else None
            out.append(MatchResult(query_idx=q, match_idx=m, num_keypoints_query=len(k1), num_keypoints_match=len(k2),
                                   num_matches=len(k1), num_inliers=n_in, inlier_ratio=ratio, relative_pose=pose,
                                   essential_matrix=E, confidence=min(1.0, ratio * (n_in / self.min_inliers)),
                                   is_valid=n_in >= self.min_inliers and ratio >= self.min_inlier_ratio))
        return out

    def verify_batch(self, image_pairs: List[Tuple[np.ndarray, np.ndarray]], K: Optional[np.ndarray] = None,
                     indices: Optional[List[Tuple[int, int]]] = None) -> List[MatchResult]:
        """Same results as verifying each pair in turn (geometric_verification.py:636-662),
        computed as one batched matching + RANSAC pass when the images share a shape
        (every matcher has a batched path: SuperPoint + LightGlue; SuperGlue and LoFTR
        through the LightGlue fallback the reference resolves them to without magicleap /
        kornia, or their native kernels when opted in)."""
        if not image_pairs:
            return []
        if len({np.shape(im) for pair in image_pairs for im in pair}) == 1:
            frames = torch.from_numpy(np.stack([np.asarray(im, np.uint8) for pair in image_pairs for im in pair]))
            frames = frames.to(torch.device(self.matcher.device))
            return self.verify_frames_batch(frames, [(2 * i, 2 * i + 1) for i in range(len(image_pairs))], K, indices)
        out = []
        for i, (a, b) in enumerate(image_pairs):
            q, mi = indices[i] if indices is not None else (i, i)
            out.append(self.verify(a, b, K, q, mi))
        return out

    def verify_frames_batch(self, frames, pairs: List[Tuple[int, int]], K: Optional[np.ndarray] = None,
                            indices: Optional[List[Tuple[int, int]]] = None) -> List[MatchResult]:
        """verify() for pairs (a, b) of device-resident keyframes frames[a], frames[b]
        (uint8 [F, H, W, C]): SuperPoint once per distinct keyframe, LightGlue over all
        pairs in one ragged call, one batched RANSAC + recoverPose, the decision rule."""
        if not pairs:
            return []
        matched = self.matcher.detect_and_match_batch(frames, pairs)
        return self.verify_matches_batch([(a, b) for a, b, _ in matched], K, indices)


class SemanticGeometricVerifier(GeometricVerifier):
    """Cross-floor pairs are rejected before any matching work is spent on them."""

    def __init__(self, matcher_type: str = 'lightglue', device: str = 'cuda', min_inliers: int = 20,
                 min_inlier_ratio: float = 0.25, enable_floor_gating: bool = True):
        super().__init__(matcher_type, device, min_inliers, min_inlier_ratio)
        self.enable_floor_gating = enable_floor_gating
        self.stats = {'verified': 0, 'skipped_floor_mismatch': 0, 'valid': 0, 'invalid': 0}

    def verify_with_semantics(self, image1: np.ndarray, image2: np.ndarray, floor1: int, floor2: int,
                              K: Optional[np.ndarray] = None, query_idx: int = 0, match_idx: int = 0) -> MatchResult:
        if self.enable_floor_gating and floor1 != floor2:
            self.stats['skipped_floor_mismatch'] += 1
            return _rejected(query_idx, match_idx)
        res = self.verify(image1, image2, K, query_idx, match_idx)
        self.stats['verified'] += 1
        self.stats['valid' if res.is_valid else 'invalid'] += 1
        return res

    def verify_with_semantics_batch(self, frames, pairs: List[Tuple[int, int]], floors: List[Tuple[int, int]],
                                    K: Optional[np.ndarray] = None,
                                    indices: Optional[List[Tuple[int, int]]] = None) -> List[MatchResult]:
        """verify_with_semantics for many pairs (a, b) of device-resident keyframes with
        their floor labels (f_a, f_b): the same skip rule, results and counters as calling
        it pair by pair in this order; the pairs that are not skipped are verified in one
        batched pass (verify_frames_batch)."""
        n = len(pairs)
        idx = list(indices) if indices is not None else [(0, 0)] * n
        skip = [self.enable_floor_gating and f1 != f2 for f1, f2 in floors]
        run = [i for i in range(n) if not skip[i]]
        res = self.verify_frames_batch(frames, [pairs[i] for i in run], K, [idx[i] for i in run])
        out = [_rejected(*idx[i]) if skip[i] else None for i in range(n)]
        for i, r in zip(run, res):
            out[i] = r
        self.stats['skipped_floor_mismatch'] += sum(skip)
        self.stats['verified'] += len(run)
        n_valid = sum(1 for r in res if r.is_valid)
        self.stats['valid'] += n_valid
        self.stats['invalid'] += len(run) - n_valid
        return out

    def get_statistics(self) -> Dict:
        total = self.stats['verified'] + self.stats['skipped_floor_mismatch']
        return {**self.stats, 'total_candidates': total,
                'skip_rate': self.stats['skipped_floor_mismatch'] / total if total > 0 else 0,
                'valid_rate': self.stats['valid'] / self.stats['verified'] if self.stats['verified'] > 0 else 0}
