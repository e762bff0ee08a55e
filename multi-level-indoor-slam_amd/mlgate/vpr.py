"""Visual place recognition: the drop-in mirror of scripts/semantic_gating/place_recognition.py.

Same class names, constructor signatures, dataclasses, return types and error
behaviour as the reference; the compute runs on the mlgate HIP kernels:

  * CricaVPR -> DINOv2 ViT-B/14 + GeM on MI355X (mlgate.vit.VitB14); ONE forward per
    keyframe feeds both the descriptor and the local-feature cache (the reference runs
    the same forward twice, place_recognition.py:765/777).
  * AnyLoc   -> the same ViT at 518^2 with mean pooling and unswapped channels
    (place_recognition.py:467-505).
  * retrieval (find_loop_closures / query / pairwise similarities / cross-correlation
    rerank) -> mlg_knn_gate / mlg_knn_query / mlg_xcorr_score.
  * MixVPR / SALAD -> the reference resolves both to a torchvision ResNet-50 GAP
    fallback (place_recognition.py:241-306, 370-378); here that network runs on the
    GPU (mlgate.resnet: Pillow-exact resize, HIP stem, MFMA bottlenecks, GAP, zero-pad).
    SALAD's native branch (DINOv2 + Sinkhorn aggregation) is opt-in: mlgate.salad.

Weights: the hub checkpoint cannot be fetched offline.  ``pretrained_path`` (or
MLGATE_DINOV2_WEIGHTS) may point at a local hub-format dinov2_vitb14 state_dict;
otherwise seeded synthetic weights are used and a warning says so.
"""
import os
import warnings
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Tuple, Union

import numpy as np

from . import _native


@dataclass
class PlaceMatch:
    """A retrieved (query, match) pair; ``is_valid`` is the floor-gate decision."""
    query_idx: int
    match_idx: int
    similarity: float
    query_timestamp: Optional[float] = None
    match_timestamp: Optional[float] = None
    is_valid: bool = True


@dataclass
class PlaceDescriptor:
    """One database entry: global descriptor plus its timestamp / floor label."""
    timestamp: float
    descriptor: np.ndarray
    image_path: Optional[str] = None
    floor_label: Optional[int] = None


def _torch():
    import torch
    return torch


def _device_frames(images, device):
    """uint8 [B, H, W, C] on the device from a device / host tensor or a list of images."""
    torch = _torch()
    if isinstance(images, torch.Tensor):
        t = images if images.dim() == 4 else images.unsqueeze(-1)
        if t.dtype != torch.uint8:
            raise ValueError("frames must be uint8")
        return t.to(device).contiguous()
    return torch.from_numpy(_as_frames(images)).to(device)


def floor_codes(labels):
    """Integer codes with the reference's equality semantics for the floor check
    ``query_floor == match_floor`` (place_recognition.py:896-899): labels that compare
    equal in Python share a code (1 and 1.0 included), every NaN gets its own code
    (NaN != NaN), None marks "no label" (has = 0)."""
    codes = np.zeros(len(labels), np.int64)
    has = np.ones(len(labels), np.uint8)
    seen = {}
    nxt = 0
    for i, f in enumerate(labels):
        if f is None:
            has[i] = 0
            continue
        if isinstance(f, (float, np.floating)) and f != f:
            codes[i] = nxt
            nxt += 1
            continue
        key = f.item() if isinstance(f, np.generic) else f
        c = seen.get(key)
        if c is None:
            c = seen[key] = nxt
            nxt += 1
        codes[i] = c
    return codes, has


def _as_frames(images):
    """List / array of HxW[xC] uint8 images (one size) -> contiguous uint8 [B, H, W, C]."""
    arrs = [np.asarray(im) for im in images]
    if not arrs:
        raise ValueError("no images")
    if any(a.shape != arrs[0].shape for a in arrs):
        raise ValueError("all images of a batch must have the same shape")
    batch = np.stack(arrs).astype(np.uint8, copy=False)
    if batch.ndim == 3:
        batch = batch[..., None]
    return np.ascontiguousarray(batch)


class BasePlaceRecognition:
    """Descriptor database + GPU retrieval shared by every VPR method."""

    def __init__(self, descriptor_dim: int = 4096, device: str = 'cuda'):
        self.descriptor_dim = descriptor_dim
        self.device = device
        self.model = None
        self.descriptors: List[PlaceDescriptor] = []

    # ---------------------------------------------------------- extraction
    def extract_descriptor(self, image: np.ndarray) -> np.ndarray:
        raise NotImplementedError

    def extract_descriptors(self, images) -> np.ndarray:
        """Batched extraction (mlgate extension): [B, D] float32."""
        return np.stack([self.extract_descriptor(im) for im in images])

    def add_image(self, image: np.ndarray, timestamp: float, floor_label: Optional[int] = None,
                  image_path: Optional[str] = None) -> PlaceDescriptor:
        entry = PlaceDescriptor(timestamp=timestamp, descriptor=self.extract_descriptor(image),
                                image_path=image_path, floor_label=floor_label)
        self.descriptors.append(entry)
        return entry

    def add_images(self, images, timestamps, floor_labels=None, image_paths=None) -> List[PlaceDescriptor]:
        """Batched add_image (mlgate extension): one device batch instead of N calls."""
        descs = self.extract_descriptors(images)
        out = []
        for i, d in enumerate(descs):
            out.append(PlaceDescriptor(timestamp=timestamps[i], descriptor=d,
                                       image_path=None if image_paths is None else image_paths[i],
                                       floor_label=None if floor_labels is None else floor_labels[i]))
        self.descriptors.extend(out)
        return out

    # ---------------------------------------------------------- database
    def build_descriptor_matrix(self) -> np.ndarray:
        if not self.descriptors:
            return np.array([])
        return np.vstack([d.descriptor for d in self.descriptors])

    def _device_matrix(self):
        """Device float32 [N, D] mirror of ``self.descriptors``.  Callers may append to (or
        replace entries of) the public list directly, as the reference allows
        (place_recognition.py:1020); the mirror tracks the descriptor arrays by identity
        and uploads only rows whose array object changed (appends upload only the new
        rows).  In-place edits of a descriptor array's values are not seen: replace the
        PlaceDescriptor (or its array) instead."""
        torch = _torch()
        dev = _native.require_device(self.device)
        arrs = [d.descriptor for d in self.descriptors]
        ids = [id(a) for a in arrs]
        m = getattr(self, '_mirror', None)
        D = int(np.asarray(arrs[0]).size) if arrs else 0
        if m is None or m['dev'] != dev or m['D'] != D or m['buf'].shape[0] < len(arrs):
            cap = max(len(arrs), 64, 0 if m is None else 2 * m['buf'].shape[0])
            buf = torch.empty(cap, D, dtype=torch.float32, device=dev)
            m = self._mirror = {'dev': dev, 'D': D, 'buf': buf, 'ids': [], 'keep': []}
        old = m['ids']
        stale = [i for i in range(len(ids)) if i >= len(old) or old[i] != ids[i]]
        if stale:
            lo = stale[0]
            if len(stale) == len(ids) - lo:  # one contiguous tail: a single upload
                rows = np.ascontiguousarray(np.stack([np.asarray(a, np.float32).reshape(-1) for a in arrs[lo:]]))
                m['buf'][lo:len(ids)].copy_(torch.from_numpy(rows))
            else:
                for i in stale:
                    m['buf'][i].copy_(torch.from_numpy(np.ascontiguousarray(arrs[i], dtype=np.float32).reshape(-1)))
        m['ids'] = ids
        m['keep'] = arrs  # hold the arrays so their ids stay unique while mirrored
        return m['buf'][:len(ids)], dev

    def compute_all_pairwise_similarities(self) -> np.ndarray:
        """N x N cosine similarities (float32), computed on the device."""
        if not self.descriptors:
            return np.array([])
        from . import retrieval
        X, _ = self._device_matrix()
        return retrieval.pairwise_similarities(X).cpu().numpy()

    def _compute_similarity(self, query: np.ndarray, database: np.ndarray) -> np.ndarray:
        torch = _torch()
        from . import retrieval
        dev = _native.require_device(self.device)
        db = torch.from_numpy(np.ascontiguousarray(database, dtype=np.float32)).to(dev)
        q = torch.from_numpy(np.ascontiguousarray(np.asarray(query, np.float32).reshape(1, -1))).to(dev)
        return retrieval.similarity(q, db)[0].cpu().numpy()

    def query(self, image: np.ndarray, timestamp: Optional[float] = None, k: int = 5,
              min_time_gap: float = 10.0) -> List[PlaceMatch]:
        """Top-k database entries for a new image (the query is not added)."""
        if not self.descriptors:
            return []
        torch = _torch()
        from . import retrieval
        qd = self.extract_descriptor(image)
        db, dev = self._device_matrix()
        t_db = torch.tensor([float(d.timestamp) for d in self.descriptors], dtype=torch.float64, device=dev)
        tq = torch.tensor([float('nan') if timestamp is None else float(timestamp)], dtype=torch.float64,
                          device=dev)
        q = torch.from_numpy(np.asarray(qd, np.float32).reshape(1, -1)).to(dev)
        kk = max(1, min(k, len(self.descriptors)))
        idx, sim, cnt = retrieval.knn_query(db, q, t_db, tq, min_time_gap if timestamp is not None else 0.0, kk)
        c = int(cnt[0]) if k > 0 else 0
        idx, sim = idx[0, :c].cpu().numpy(), sim[0, :c].cpu().numpy()
        n = len(self.descriptors)
        return [PlaceMatch(query_idx=n, match_idx=int(j), similarity=float(s), query_timestamp=timestamp,
                           match_timestamp=self.descriptors[int(j)].timestamp) for j, s in zip(idx, sim)]


class _ResNetFallback(BasePlaceRecognition):
    """MixVPR / SALAD: what the reference executes is a torchvision ResNet-50 GAP
    (place_recognition.py:248-306) -- the MixVPR / SALAD packages are never importable
    under the names it tries, so every call lands in ``_load_fallback_model``.  Here
    that network runs on the GPU (mlgate.resnet, HIP kernels + bf16 MFMA GEMMs)."""

    def __init__(self, descriptor_dim, device, pretrained_path=None):
        super().__init__(descriptor_dim, device)
        self.pretrained_path = pretrained_path
        self._model_loaded = False

    def _load_model(self):
        if self._model_loaded:
            return
        from .resnet import ResNet50GPU
        self._net = ResNet50GPU(device=self.device)
        if self._net.weights_source.startswith("synthetic"):
            warnings.warn("ImageNet ResNet-50 weights are not available offline; using seeded synthetic resnet50 "
                          "weights (set MLGATE_RESNET50_WEIGHTS to a local torchvision checkpoint).")
        self._model_loaded = True
        self._is_fallback = True

    def extract_descriptors(self, images) -> np.ndarray:
        self._load_model()
        frames = _device_frames(images, self._net.device)
        return self._net.forward_device(frames, self.descriptor_dim).cpu().numpy()

    def extract_descriptor(self, image: np.ndarray) -> np.ndarray:
        return self.extract_descriptors([image])[0]


class MixVPR(_ResNetFallback):
    def __init__(self, backbone: str = 'resnet50', descriptor_dim: int = 4096, device: str = 'cuda',
                 pretrained_path: Optional[str] = None):
        super().__init__(descriptor_dim, device, pretrained_path)
        self.backbone_name = backbone


class SALAD(_ResNetFallback):
    """place_recognition.py:335-410.  By default what the reference executes: the
    ``salad`` package does not import, so SALAD warns and runs the MixVPR fallback
    (:370-378).  ``MLGATE_SALAD_NATIVE=1`` (or ``.native = True``) selects the model its
    native branch names (:357-368): serizba/salad's DINOv2 ViT-B/14 + optimal-transport
    aggregator (64 clusters x 128 + 256 token dims = 8448) on the GPU (mlgate.salad,
    csrc/salad.hip); weights from ``pretrained_path`` / MLGATE_SALAD_WEIGHTS, else seeded
    synthetic ones."""

    def __init__(self, descriptor_dim: int = 8448, device: str = 'cuda', pretrained_path: Optional[str] = None):
        super().__init__(descriptor_dim, device, pretrained_path)
        self.native = None  # None: MLGATE_SALAD_NATIVE decides; True / False force it
        self._salad = None

    def _load_model(self):
        if self._model_loaded:
            return
        native = self.native if self.native is not None else os.environ.get("MLGATE_SALAD_NATIVE") == "1"
        if not native:
            warnings.warn("SALAD not installed. Using MixVPR fallback. For SALAD: pip install salad-vpr")
            return super()._load_model()
        from .salad import DESC_DIM, SaladGPU
        if self.descriptor_dim != DESC_DIM:
            raise ValueError(f"native SALAD produces {DESC_DIM}-dim descriptors, not {self.descriptor_dim}")
        self._salad = SaladGPU(device=self.device, pretrained_path=self.pretrained_path)
        if self._salad.weights_source.startswith("synthetic"):
            warnings.warn("SALAD weights not configured (pretrained_path / MLGATE_SALAD_WEIGHTS); using seeded "
                          "synthetic weights")
        self._model_loaded = True
        self._is_fallback = False

    def extract_descriptors(self, images) -> np.ndarray:
        self._load_model()
        if self._salad is None:
            return super().extract_descriptors(images)
        return self._salad.forward(_device_frames(images, self._salad.device)).cpu().numpy()


class _DinoEngineMixin:
    """Lazy ViT-B/14 engine construction shared by CricaVPR and AnyLoc."""

    _image_size = 322
    _pool = "gem"
    _swap_rb = True

    def _engine(self):
        if getattr(self, '_vit', None) is None:
            if self.backbone_name != 'dinov2_vitb14':
                raise ValueError(f"{self.backbone_name}: only the dinov2_vitb14 backbone has MI355X kernels")
            from .vit import VitB14
            from .weights import resolve_state_dict
            sd, source = resolve_state_dict(getattr(self, 'pretrained_path', None))
            if source.startswith('synthetic'):
                warnings.warn("DINOv2 hub weights are not available offline; using seeded synthetic "
                              "dinov2_vitb14 weights (set pretrained_path or MLGATE_DINOV2_WEIGHTS to a local "
                              "hub checkpoint for real descriptors).")
            # the split-bf16 forward (VitB14's default): descriptors within ~1e-11 of fp32,
            # so retrieval ranks as the fp32 reference does
            self._vit = VitB14(sd, device=self.device, image_size=self._image_size, pool=self._pool,
                               swap_rb=self._swap_rb, precise=True)
            self.feat_dim = 768
            self._model_loaded = True
        return self._vit

    def _forward(self, images, with_local=False):
        eng = self._engine()
        return eng.forward(_device_frames(images, eng.device), with_local=with_local)

    def extract_descriptors(self, images) -> np.ndarray:
        return self._forward(images).cpu().numpy()

    def extract_descriptor(self, image: np.ndarray) -> np.ndarray:
        return self._forward([image])[0].cpu().numpy().flatten()


class AnyLoc(_DinoEngineMixin, BasePlaceRecognition):
    _image_size = 518
    _pool = "mean"
    _swap_rb = False

    def __init__(self, backbone: str = 'dinov2_vitb14', descriptor_dim: int = 49152, device: str = 'cuda',
                 num_clusters: int = 64):
        super().__init__(descriptor_dim, device)
        self.backbone_name = backbone
        self.num_clusters = num_clusters
        self._model_loaded = False
        self._vit = None


class CricaVPR(_DinoEngineMixin, BasePlaceRecognition):
    def __init__(self, backbone: str = 'dinov2_vitb14', descriptor_dim: int = 10752, device: str = 'cuda',
                 pretrained_path: Optional[str] = None, use_reranking: bool = True):
        super().__init__(descriptor_dim, device)
        self.backbone_name = backbone
        self.pretrained_path = pretrained_path
        self.use_reranking = use_reranking
        self._model_loaded = False
        self._vit = None
        self._feature_cache = {}  # idx -> device float32 [1, 528, 768]

    def extract_local_features(self, image: np.ndarray) -> np.ndarray:
        _, local = self._forward([image], with_local=True)
        return local.cpu().numpy()

    def _to_device_feats(self, f):
        torch = _torch()
        dev = self._engine().device if getattr(self, '_vit', None) is not None else _native.require_device(
            self.device)
        t = f if isinstance(f, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(f, dtype=np.float32))
        t = t.to(dev, torch.float32)
        if t.dim() == 3:
            t = t.squeeze(0)
        return t.contiguous()

    def compute_cross_correlation_score(self, query_features, match_features) -> float:
        from . import retrieval
        return float(retrieval.xcorr_score(self._to_device_feats(query_features),
                                           self._to_device_feats(match_features)).item())

    def rerank_candidates(self, query_idx: int, candidates: List[Tuple[int, float]],
                          top_k: int = 5) -> List[Tuple[int, float]]:
        """place_recognition.py:714-757: 0.5 global + 0.5 cross-correlation, sorted
        (stable) by the combined score; every candidate of the query scored in ONE batched
        pass (mlg_xcorr_batch) instead of one correlation per candidate."""
        if not self.use_reranking or query_idx not in self._feature_cache:
            return candidates[:top_k]
        return self.rerank_candidates_batch({query_idx: candidates}, top_k)[query_idx]

    def rerank_candidates_batch(self, requests: Dict[int, List[Tuple[int, float]]],
                                top_k: int = 5) -> Dict[int, List[Tuple[int, float]]]:
        """rerank_candidates for many queries at once ({query_idx: [(match_idx,
        global_sim), ...]}): all (query, candidate) cross-correlation scores of all
        queries in one batched pass over the cached local features (one frame bank, no
        [L, L] matrix per pair), then the reference's combination and stable sort per query."""
        torch = _torch()
        pairs = [(q, j) for q, cands in requests.items() if self.use_reranking and q in self._feature_cache
                 for j, _ in cands if j in self._feature_cache]
        scores = {}
        if pairs:
            frames = sorted({i for p in pairs for i in p})
            pos = {f: k for k, f in enumerate(frames)}
            bank = torch.cat([self._to_device_feats(self._feature_cache[f])[None] for f in frames])
            dev = bank.device
            qa = torch.tensor([pos[q] for q, _ in pairs], dtype=torch.int32, device=dev)
            qb = torch.tensor([pos[j] for _, j in pairs], dtype=torch.int32, device=dev)
            sc = _native.ops().xcorr_batch(bank.contiguous(), qa, qb).cpu().numpy()
            scores = {p: float(v) for p, v in zip(pairs, sc)}
        out = {}
        for q, cands in requests.items():
            if not self.use_reranking or q not in self._feature_cache:
                out[q] = cands[:top_k]
                continue
            scored = [(j, 0.5 * g + 0.5 * scores[(q, j)]) if (q, j) in scores else (j, g) for j, g in cands]
            scored.sort(key=lambda x: x[1], reverse=True)
            out[q] = scored[:top_k]
        return out

    def _append(self, descs, local, timestamps, floor_labels, image_paths):
        out = []
        for i in range(len(descs)):
            entry = PlaceDescriptor(timestamp=timestamps[i], descriptor=descs[i],
                                    image_path=None if image_paths is None else image_paths[i],
                                    floor_label=None if floor_labels is None else floor_labels[i])
            self.descriptors.append(entry)
            if self.use_reranking:
                self._feature_cache[len(self.descriptors) - 1] = local[i:i + 1]
            out.append(entry)
        return out

    def add_image(self, image: np.ndarray, timestamp: float, floor_label: Optional[int] = None,
                  image_path: Optional[str] = None) -> PlaceDescriptor:
        desc, local = self._forward([image], with_local=True)
        return self._append(desc.cpu().numpy(), local, [timestamp], [floor_label], [image_path])[0]

    def add_images(self, images, timestamps, floor_labels=None, image_paths=None) -> List[PlaceDescriptor]:
        desc, local = self._forward(images, with_local=True)
        return self._append(desc.cpu().numpy(), local, timestamps, floor_labels, image_paths)


_METHODS = {'mixvpr': MixVPR, 'salad': SALAD, 'anyloc': AnyLoc, 'cricavpr': CricaVPR}


class SemanticPlaceRecognition:
    """VPR database + floor-gated all-keyframes loop-closure retrieval."""

    def __init__(self, vpr_method: str = 'mixvpr', device: str = 'cuda', similarity_threshold: float = 0.5,
                 min_time_gap: float = 10.0):
        self.similarity_threshold = similarity_threshold
        self.min_time_gap = min_time_gap
        key = vpr_method.lower()
        if key not in _METHODS:
            raise ValueError(f"Unknown VPR method: {vpr_method}. Available: mixvpr, salad, anyloc, cricavpr")
        self.vpr = CricaVPR(device=device, use_reranking=True) if key == 'cricavpr' else _METHODS[key](device=device)

    def add_image(self, image: np.ndarray, timestamp: float, floor_label: int,
                  image_path: Optional[str] = None) -> PlaceDescriptor:
        return self.vpr.add_image(image, timestamp, floor_label, image_path)

    def add_images(self, images, timestamps, floor_labels, image_paths=None) -> List[PlaceDescriptor]:
        """Batched add_image (mlgate extension)."""
        return self.vpr.add_images(images, timestamps, floor_labels, image_paths)

    def find_loop_closures(self, enable_floor_gating: bool = True, k: int = 10) -> List[PlaceMatch]:
        descs = self.vpr.descriptors
        n = len(descs)
        if n < 2:
            return []
        torch = _torch()
        from . import retrieval
        if k <= 0:
            return []
        # a row ranks all n entries (its own included when min_time_gap <= 0): k beyond n
        # returns what argsort()[:k] returns, every candidate
        kk = min(k, n)
        X, dev = self.vpr._device_matrix()
        t = torch.tensor([float(d.timestamp) for d in descs], dtype=torch.float64, device=dev)
        codes, has = floor_codes([d.floor_label for d in descs])
        fl = torch.from_numpy(codes).to(dev)
        hf = torch.from_numpy(has).to(dev)
        out = retrieval.knn_gate(X, t, fl, hf, self.min_time_gap, self.similarity_threshold, kk,
                                 enable_floor_gating)
        q, m, sim, valid = retrieval.flatten_matches(*out)
        return [PlaceMatch(query_idx=int(i), match_idx=int(j), similarity=float(s),
                           query_timestamp=descs[int(i)].timestamp, match_timestamp=descs[int(j)].timestamp,
                           is_valid=bool(v)) for i, j, s, v in zip(q, m, sim, valid)]

    def get_statistics(self, matches: List[PlaceMatch]) -> Dict:
        if not matches:
            return {'total_matches': 0, 'valid_matches': 0, 'rejected_matches': 0, 'rejection_rate': 0.0}
        ok = [m.is_valid for m in matches]
        n_valid = sum(ok)
        n = len(matches)
        sims = [m.similarity for m in matches]
        return {
            'total_matches': n,
            'valid_matches': n_valid,
            'rejected_matches': n - n_valid,
            'rejection_rate': (n - n_valid) / n,
            'mean_similarity': np.mean(sims),
            'mean_valid_similarity': np.mean([s for s, v in zip(sims, ok) if v]) if n_valid > 0 else 0.0,
        }


def process_image_sequence(image_dir: Union[str, Path], timestamps: np.ndarray, floor_labels: np.ndarray,
                           vpr_method: str = 'mixvpr',
                           device: str = 'cuda') -> Tuple[SemanticPlaceRecognition, List[PlaceMatch]]:
    """Sorted *.png then *.jpg of a directory -> database -> floor-gated loop closures
    (place_recognition.py:936-991).

    PNG keyframes (what bag_utils.extract_images writes) are decoded by the native
    loader (mlgate.ingest: host thread pool -> pinned buffer -> HBM on a side stream)
    and added in device batches; the database, warnings and matches are those of the
    reference's one-image-at-a-time loop.  *.jpg files go through cv2.imread when OpenCV is
    installed, else through Pillow's libjpeg(-turbo) decode (mlgate.ingest.jpeg_reader)."""
    from . import ingest
    image_dir = Path(image_dir)
    spr = SemanticPlaceRecognition(vpr_method=vpr_method, device=device)
    files = sorted(image_dir.glob('*.png')) + sorted(image_dir.glob('*.jpg'))
    if len(files) != len(timestamps):
        warnings.warn(f"Number of images ({len(files)}) != timestamps ({len(timestamps)}). Using minimum of both.")
    n = min(len(files), len(timestamps), len(floor_labels))
    files = files[:n]
    jpeg_read = None
    if any(f.suffix == '.jpg' for f in files):
        jpeg_read = ingest.jpeg_reader()  # cv2.imread, else Pillow's libjpeg decode; ImportError if neither
    print(f"Processing {n} images with {vpr_method}...")
    pngs = [i for i, f in enumerate(files) if f.suffix == '.png']
    for idx, frames in ingest.KeyframeStream([files[i] for i in pngs], device=device):
        rows = [pngs[j] for j in idx]
        spr.add_images(frames, [timestamps[i] for i in rows], [int(floor_labels[i]) for i in rows],
                       [str(files[i]) for i in rows])
        for i in rows:
            if (i + 1) % 100 == 0:
                print(f"  Processed {i + 1}/{n} images")
    for i in range(len(pngs), n):  # *.jpg files sort after every *.png file
        img = jpeg_read(files[i])
        if img is None:
            warnings.warn(f"Failed to load image: {files[i]}")
            continue
        spr.add_image(image=img, timestamp=timestamps[i], floor_label=int(floor_labels[i]), image_path=str(files[i]))
        if (i + 1) % 100 == 0:
            print(f"  Processed {i + 1}/{n} images")
    print("Finding loop closure candidates...")
    return spr, spr.find_loop_closures(enable_floor_gating=True)
