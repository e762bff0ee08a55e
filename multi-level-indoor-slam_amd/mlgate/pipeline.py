"""The full semantic loop-closure gate (BASELINE configs[3]).

No reference module chains the gate's stages; SURVEY.md §3.5 defines the harness from
the reference's public APIs, and this module is that harness:

  1. floor labels  IMUFloorDetector.detect_elevator_events / assign_floor_labels
                   (floor_detector.py:63-156), or labels given per keyframe;
  2. descriptors   SemanticPlaceRecognition('cricavpr').add_image per keyframe
                   (place_recognition.py:843-849; here one batched add_images);
  3. retrieval     find_loop_closures(enable_floor_gating, k) (:851-911);
  4. verification  SemanticGeometricVerifier.verify_with_semantics on every retrieved
                   match with is_valid (geometric_verification.py:688-734; batched);
  5. gate          SemanticLoopClosureGate(floor_labels).gate_candidates on the
                   geometrically valid pairs (loop_closure_gate.py:105-126).

The false-loop-closure rejection count is the sum of four terms:
retrieval matches with PlaceMatch.is_valid False (place_recognition.py:896-899),
verifier skips on a floor mismatch (geometric_verification.py:709-710), verifier
invalid results (:729-732) and the gate's rejected_cross_floor (loop_closure_gate.py:
91-98).

Two front ends run the same kernels:
  * ``FullSemanticGate`` composes the drop-in classes (PlaceMatch / MatchResult /
    LoopClosureCandidate objects, the reference's stats dicts);
  * ``DeviceGate`` is the same chain on device arrays, frame-sharded over ranks (one
    process per GPU, RCCL all-gathers; bench.py's step).  Its decisions and counts are
    those of FullSemanticGate (tests/test_pipeline_gpu.py).
"""
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import _native

from .floors import IMUFloorDetector
from .gate import LoopClosureCandidate, SemanticLoopClosureGate
from .verify import MatchResult, SemanticGeometricVerifier
from .vpr import PlaceMatch, SemanticPlaceRecognition


@dataclass
class RejectionCount:
    """The four terms of the false-loop-closure rejection count."""
    retrieval_floor_rejected: int = 0   # PlaceMatch.is_valid == False
    skipped_floor_mismatch: int = 0     # SemanticGeometricVerifier skip branch
    verifier_invalid: int = 0           # geometric verification failed
    gate_rejected_cross_floor: int = 0  # SemanticLoopClosureGate rejections

    @property
    def total(self) -> int:
        return (self.retrieval_floor_rejected + self.skipped_floor_mismatch + self.verifier_invalid
                + self.gate_rejected_cross_floor)

    def as_dict(self) -> Dict[str, int]:
        return {'retrieval_floor_rejected': self.retrieval_floor_rejected,
                'skipped_floor_mismatch': self.skipped_floor_mismatch,
                'verifier_invalid': self.verifier_invalid,
                'gate_rejected_cross_floor': self.gate_rejected_cross_floor, 'total': self.total}


@dataclass
class GateReport:
    floor_labels: np.ndarray
    events: list
    matches: List[PlaceMatch]
    verified: List[PlaceMatch]          # matches sent to the verifier, in emission order
    results: List[MatchResult]          # one per verified match
    accepted: List[LoopClosureCandidate]
    rejected: List[LoopClosureCandidate]
    retrieval_stats: Dict
    verifier_stats: Dict
    gate_stats: Dict
    rejections: RejectionCount = field(default_factory=RejectionCount)


def floor_labels_from_imu(timestamps, imu, start_floor=5, detector_kwargs=None):
    """(labels, events) from an IMU log (t, ax, ay, az) -- floor_detector.py:63-156."""
    det = IMUFloorDetector(**(detector_kwargs or {}))
    t, ax, ay, az = imu[:4]
    events = det.detect_elevator_events(np.asarray(t), np.asarray(ax), np.asarray(ay), np.asarray(az))
    return det.assign_floor_labels(np.asarray(timestamps), start_floor=start_floor), events


class FullSemanticGate:
    """IMU floors -> CricaVPR descriptors -> floor-gated kNN -> semantic geometric
    verification -> floor gate, composed from the drop-in API."""

    def __init__(self, vpr_method: str = 'cricavpr', matcher_type: str = 'lightglue', device: str = 'cuda',
                 similarity_threshold: float = 0.5, min_time_gap: float = 10.0, k: int = 10, min_inliers: int = 20,
                 min_inlier_ratio: float = 0.25, strict_mode: bool = True, retrieval_floor_gating: bool = True,
                 verifier_floor_gating: bool = True, verify_rejected: bool = False, start_floor: int = 5,
                 imu_detector_kwargs: Optional[Dict] = None):
        self.vpr_method, self.matcher_type, self.device = vpr_method, matcher_type, device
        self.similarity_threshold, self.min_time_gap, self.k = similarity_threshold, min_time_gap, k
        self.min_inliers, self.min_inlier_ratio, self.strict_mode = min_inliers, min_inlier_ratio, strict_mode
        self.retrieval_floor_gating = retrieval_floor_gating
        self.verifier_floor_gating = verifier_floor_gating
        self.verify_rejected = verify_rejected  # also send is_valid == False matches to the verifier
        self.start_floor = start_floor
        self.imu_detector_kwargs = imu_detector_kwargs
        self.spr = None
        self.verifier = None
        self.gate = None

    def run(self, images, timestamps, K: Optional[np.ndarray] = None, floor_labels=None, imu=None) -> GateReport:
        """images: uint8 [N, H, W, C] device tensor or N numpy images; timestamps [N];
        floor labels given, or derived from ``imu`` = (t, ax, ay, az)."""
        import torch
        timestamps = np.asarray(timestamps, np.float64)
        events = []
        if floor_labels is None:
            if imu is None:
                raise ValueError("need floor_labels or an IMU log")
            floor_labels, events = floor_labels_from_imu(timestamps, imu, self.start_floor, self.imu_detector_kwargs)
        floor_labels = np.asarray(floor_labels)
        self.spr = SemanticPlaceRecognition(self.vpr_method, self.device, self.similarity_threshold,
                                            self.min_time_gap)
        if isinstance(images, torch.Tensor):
            frames = images
        else:
            frames = torch.from_numpy(np.ascontiguousarray(np.stack([np.asarray(im, np.uint8) for im in images])))
        frames = frames.to(torch.device(self.device))
        labels = [int(f) if np.issubdtype(type(f), np.integer) else f for f in floor_labels.tolist()]
        self.spr.add_images(frames, timestamps.tolist(), labels)
        matches = self.spr.find_loop_closures(enable_floor_gating=self.retrieval_floor_gating, k=self.k)
        to_verify = [m for m in matches if m.is_valid or self.verify_rejected]
        self.verifier = SemanticGeometricVerifier(self.matcher_type, self.device, self.min_inliers,
                                                  self.min_inlier_ratio, enable_floor_gating=self.verifier_floor_gating)
        pairs = [(m.query_idx, m.match_idx) for m in to_verify]
        results = self.verifier.verify_with_semantics_batch(frames, pairs,
                                                            [(labels[a], labels[b]) for a, b in pairs], K, pairs)
        self.gate = SemanticLoopClosureGate(floor_labels, strict_mode=self.strict_mode)
        accepted, rejected = self.gate.gate_candidates(
            [(m.query_idx, m.match_idx, m.similarity) for m, r in zip(to_verify, results) if r.is_valid])
        vstats = self.verifier.get_statistics()
        gstats = self.gate.get_stats()
        counts = RejectionCount(retrieval_floor_rejected=sum(1 for m in matches if not m.is_valid),
                                skipped_floor_mismatch=vstats['skipped_floor_mismatch'],
                                verifier_invalid=vstats['invalid'],
                                gate_rejected_cross_floor=gstats['rejected_cross_floor'])
        return GateReport(floor_labels=floor_labels, events=events, matches=matches, verified=to_verify,
                          results=results, accepted=accepted, rejected=rejected,
                          retrieval_stats=self.spr.get_statistics(matches), verifier_stats=vstats,
                          gate_stats=gstats, rejections=counts)


class DeviceGate:
    """The same chain on device arrays for a frame-sharded sequence: rank r of W owns
    keyframes [r N / W, (r + 1) N / W) -- its frames, ViT forwards and SuperPoint
    features -- and the query rows of the same range.  Exchange steps (RCCL over
    xGMI; gloo through host copies): the [N, 768] descriptor all-gather before retrieval,
    an 8-B-per-pair all-gather that re-balances the gate-accepted pairs across ranks
    (mlgate.distributed.balanced_pairs), and the SuperPoint features of exactly the
    keyframes each rank's pair slice touches (mlgate.distributed.FeatureExchange).

    One ``step()`` gates the whole sequence once and returns per-rank counts; the
    caller all-reduces them (bench.py)."""

    def __init__(self, frames, timestamps, floor_labels, world=1, rank=0, device='cuda', k=10,
                 similarity_threshold=0.5, min_time_gap=10.0, strict_mode=True, retrieval_floor_gating=True,
                 verifier_floor_gating=True, verify=True, K=None, min_inliers=20, min_inlier_ratio=0.25,
                 vit_batch=123, sp_batch=64, lg_chunk=1024, max_keypoints=2048, vit_state_dict=None, record=False,
                 vit_precise=True, matcher='lightglue', loftr_chunk=256, max_pairs=None, lg_tail=0,
                 local_features=True):
        import torch
        from . import distributed as mdist
        from .lightglue import LightGlueGPU
        from .superpoint import SuperPointGPU
        from .vit import VitB14
        from .weights import EMBED, synthetic_state_dict
        self.torch, self.mdist = torch, mdist
        self.dev = torch.device(device)
        self.world, self.rank = world, rank
        N = self.N = len(timestamps)
        self.lo, self.hi = mdist.shard(N, world, rank)
        self.n_local = self.hi - self.lo
        if frames.shape[0] != self.n_local:
            raise ValueError(f"rank {rank} owns {self.n_local} keyframes, got {frames.shape[0]} frames")
        self.frames = frames
        self.k, self.thr, self.gap = int(k), float(similarity_threshold), float(min_time_gap)
        self.limit = 0 if strict_mode else 1
        self.retrieval_floor_gating, self.verifier_floor_gating = retrieval_floor_gating, verifier_floor_gating
        self.min_inliers, self.min_inlier_ratio = min_inliers, min_inlier_ratio
        # lg_chunk: pairs per LightGlue call, or 'auto' (sized from the free HBM when the pairs
        # are known: _lg_chunk_for)
        self.sp_batch, self.lg_chunk, self.kp = sp_batch, lg_chunk, max_keypoints
        self.lg_tail = int(lg_tail)
        self.t_all = torch.as_tensor(np.asarray(timestamps, np.float64), device=self.dev)
        from .vpr import floor_codes
        self.labels = np.asarray(floor_labels)
        # equality codes for the retrieval floor check and the verifier skip (Python ==
        # semantics: 1 == 1.0, NaN != NaN, None = no label), the numeric labels for the
        # gate's |floor_i - floor_j| > limit (loop_closure_gate.py:91-98; NaN never rejects)
        lab = list(self.labels.tolist()) if self.labels.dtype != object else list(self.labels)
        codes, has = floor_codes(lab)
        self.h_codes, self.h_has = np.asarray(codes), np.asarray(has, np.uint8)
        self.f_all = torch.as_tensor(codes, device=self.dev)
        self.hf_all = torch.as_tensor(has, dtype=torch.uint8, device=self.dev)
        num = np.array([np.nan if v is None else float(v) for v in lab], np.float64)
        self.f_num = torch.as_tensor(num, device=self.dev)
        sd = vit_state_dict if vit_state_dict is not None else synthetic_state_dict(0)
        # vit_precise: the split-bf16 ViT (MLG_VIT_SPLIT), whose descriptors follow the fp32
        # network closely enough that the kNN ranks near-ties as the fp32 reference does
        self.eng = VitB14(sd, device=self.dev, max_batch=vit_batch, precise=vit_precise)
        self.gather = mdist.RowGather(N, EMBED, world, self.dev)
        self.desc_loc = (self.gather.out[self.lo:self.hi] if world == 1
                         else torch.empty(self.n_local, EMBED, device=self.dev))
        # CricaVPR's per-keyframe local features (place_recognition.py:645-667, the input of
        # rerank_candidates), written by the same ViT forward: [N, 528, 768] f32, 1.6 MB per
        # keyframe.  local_features=False leaves them unmaterialised (the gate itself never
        # reads them): the N = 19,163 sequence then fits one GPU with its LightGlue workspace
        self.local_feats = (torch.empty(self.n_local, self.eng.n_local, EMBED, dtype=torch.float32, device=self.dev)
                            if local_features else None)
        self.totals = torch.zeros(2, dtype=torch.int64, device=self.dev)
        self.verify = verify
        # matcher: 'lightglue' (SuperPoint + LightGlue, the reference default) or 'loftr'
        # (GeometricVerifier('loftr'), geometric_verification.py:424-526; BASELINE configs[4])
        if matcher not in ('lightglue', 'loftr'):
            raise ValueError(f"Unknown matcher: {matcher}")
        self.matcher = matcher
        self.loftr_chunk = int(loftr_chunk)
        self.max_pairs = max_pairs  # verify only the first max_pairs pairs of the global list (bench sub-runs)
        if verify and matcher == 'loftr':
            from .loftr import LoFTRGPU
            self.lf = LoFTRGPU(device=self.dev, feature_batch=16)
            self.fx = mdist.FeatureExchange(N, world, rank) if world > 1 else None
            Kc = np.asarray(K if K is not None else np.eye(3), np.float64)
            self.K = torch.from_numpy(Kc.reshape(9).copy()).to(self.dev) if K is not None else None
        elif verify:
            KP = max_keypoints
            self.sp = SuperPointGPU(device=self.dev, max_num_keypoints=KP)
            self.lg = LightGlueGPU(device=self.dev)
            # this rank's keyframes' features; with world > 1 each rank then receives the
            # features of exactly the keyframes its verification slice touches
            self.kp_loc = torch.empty(self.n_local, KP * 2, device=self.dev)
            self.ds_loc = torch.empty(self.n_local, KP * 256, device=self.dev)
            # zeros: with the SuperPoint overlap the first chunk's call sees rows not yet
            # extracted this step, and mlg_lightglue range-checks every count
            self.cnt_loc = torch.zeros(self.n_local, 1, dtype=torch.int32, device=self.dev)
            self.fx = mdist.FeatureExchange(N, world, rank) if world > 1 else None
            Kc = np.asarray(K if K is not None else np.eye(3), np.float64)
            self.K = torch.from_numpy(Kc.reshape(9).copy()).to(self.dev) if K is not None else None
        self.last = {}
        # record=True: step() keeps every verified ordered pair's (a, b, matches, inliers,
        # is_valid) in self.last_pair_results (host arrays in verification order)
        self.record = record
        # time_verify=True: _verify_loftr brackets its work with device syncs and leaves the
        # wall time in last_verify_s (bench.py's LoFTR sub-run); off, the gate never syncs for it
        self.time_verify = False
        self.last_verify_s = None
        self.last_pair_results = None
        self.last_retrieval = None

    def _dedup(self):
        """Match each unordered pair once (MLGATE_LG_DEDUP=0: every ordered pair, for A/B)."""
        import os
        return os.environ.get("MLGATE_LG_DEDUP", "1") != "0"

    def _side_stream(self):
        """The RANSAC stream (MLGATE_RANSAC_SIDE=0: the main stream, for A/B runs)."""
        if getattr(self, "_side", None) is None:
            import os
            same = os.environ.get("MLGATE_RANSAC_SIDE", "1") == "0"
            self._side = (self.torch.cuda.current_stream(self.dev) if same
                          else self.torch.cuda.Stream(device=self.dev))
        return self._side

    def step(self):
        """Gate the sequence once.  Returns this rank's counts (dict of ints): matches,
        the four rejection terms, pairs verified, pairs geometrically valid, accepted.
        The step's own work runs on a high-priority stream, so the hardware dispatches its
        workgroups ahead of the side streams' (RANSAC, SuperPoint): they fill the gaps and
        kernel tails instead of taking CUs from the LightGlue kernels (same-box A/B,
        profiles/r06p_ab_main_priority.txt: attention -2 % per launch, step time equal).
        MLGATE_MAIN_PRIORITY=0: everything at normal priority (A/B)."""
        import os
        if os.environ.get("MLGATE_MAIN_PRIORITY", "1") != "1":
            return self._step()
        torch = self.torch
        if getattr(self, "_hi", None) is None:
            self._hi = torch.cuda.Stream(device=self.dev, priority=-1)
        cur = torch.cuda.current_stream(self.dev)
        self._hi.wait_stream(cur)
        with torch.cuda.stream(self._hi):
            out = self._step()
        cur.wait_stream(self._hi)
        return out

    def _step(self):
        torch = self.torch
        from . import geometry, retrieval
        # SuperPoint of every local keyframe on its side stream (normal priority) while the
        # ViT and the kNN run on this one (high priority): it fills the ViT kernels' tails and
        # the CUs its LayerNorm / attention launches leave free (same-box ABAB, profiles/
        # r06u_ab_sp_under_vit.txt: -0.4 % step time, counts identical).  The LightGlue stage
        # waits on its event.  MLGATE_SP_UNDER_VIT=0: SuperPoint after them on this stream.
        sp_ev = None
        if self.verify and self.matcher == 'lightglue' and os.environ.get("MLGATE_SP_UNDER_VIT", "1") == "1":
            sp_ev = self._extract_side(np.arange(self.n_local))
        self.eng.forward_into(self.frames, self.desc_loc, self.local_feats)
        if self.world > 1:
            self.gather(self.desc_loc)  # RCCL all-gather of the descriptors over xGMI
        self.totals.zero_()
        idx, sim, valid, count = retrieval.knn_gate(self.gather.out, self.t_all, self.f_all, self.hf_all, self.gap,
                                                    self.thr, self.k, self.retrieval_floor_gating, q0=self.lo,
                                                    Q=self.n_local, totals=self.totals)
        # the retrieval lists come to the host once (Q x k entries): the pair list that
        # drives the verifier's chunks is built there, with no further device syncs
        h_idx, h_valid, h_count = (x.cpu().numpy() for x in (idx, valid, count))
        if self.record:  # this rank's query rows: idx / sim / valid [Q, k], count [Q] (host)
            self.last_retrieval = (h_idx, sim.cpu().numpy(), h_valid, h_count)
        k = idx.shape[1]
        live = np.arange(k)[None, :] < h_count[:, None]
        out = {"matches": int(h_count.sum()), "retrieval_floor_rejected": 0, "skipped_floor_mismatch": 0,
               "verifier_invalid": 0, "gate_rejected_cross_floor": 0, "pairs_verified": 0, "verified_valid": 0,
               "accepted": 0}
        # PlaceMatch.is_valid == False: emitted but floor-rejected
        out["retrieval_floor_rejected"] = int((live & (h_valid == 0)).sum())
        if not self.verify:
            return out
        # SuperPoint once per keyframe (the reference re-extracts per pair), cached in HBM.
        # MLGATE_SP_OVERLAP=1 (one rank): only the keyframes of the first LightGlue chunk
        # are extracted up front, the rest on a side stream under that chunk
        # (_verify_lightglue).  Same results, +0.2 % on the bench -- the LightGlue tile
        # leaves SuperPoint's convolutions little room on a CU -- while the bench's
        # per-stage HIP-event table would then time SuperPoint's launches with the
        # concurrent LightGlue in them (profiles/r05p_ab_superpoint_overlap.txt): off by
        # default.  Several ranks: all keyframes first (FeatureExchange ships finished rows).
        self._sp_overlap = (sp_ev is None and self.world == 1 and self.matcher == 'lightglue'
                            and os.environ.get("MLGATE_SP_OVERLAP", "0") == "1")
        if sp_ev is not None:
            torch.cuda.current_stream(self.dev).wait_event(sp_ev)
        elif self.matcher == 'lightglue' and not self._sp_overlap:
            self._extract_rows(np.arange(self.n_local))
        # matches handed to verify_with_semantics (is_valid ones), skip rule on floors
        qs, js = np.nonzero(live & (h_valid != 0))
        pa_h, pb_h = (qs + self.lo).astype(np.int32), h_idx[qs, js].astype(np.int32)
        if self.verifier_floor_gating:
            # verify_with_semantics skips when floor1 != floor2 in Python
            # (geometric_verification.py:709-710): None == None only, NaN != NaN
            ha, hb = self.h_has[pa_h] != 0, self.h_has[pb_h] != 0
            same = (ha & hb & (self.h_codes[pa_h] == self.h_codes[pb_h])) | (~ha & ~hb)
            out["skipped_floor_mismatch"] = int((~same).sum())
            pa_h, pb_h = pa_h[same], pb_h[same]
        pa_t, pb_t = torch.from_numpy(pa_h).to(self.dev), torch.from_numpy(pb_h).to(self.dev)
        if self.matcher == 'loftr':
            return self._verify_loftr(pa_t, pb_t, out)
        # pair-level load balance across ranks: the pairs are re-balanced first (the union
        # of the slices is the global pair list), then FeatureExchange delivers each rank
        # exactly the SuperPoint features its own slice touches
        dedup = self._dedup()
        if self.world > 1:
            pa_t, pb_t = self.mdist.balanced_pairs(pa_t, pb_t, self.world, self.rank, group_reverse=dedup)
            pa, pb = pa_t.cpu().numpy(), pb_t.cpu().numpy()
        else:
            pa, pb = pa_h, pb_h
        return self._verify_lightglue(pa, pb, dedup, out)

    def _extract_rows(self, rows):
        """SuperPoint of the local keyframes `rows` (host int array, any order) into the
        feature tables, in batches of sp_batch on the current stream.  Per-frame results do
        not depend on which frames share a batch."""
        torch = self.torch
        for b0 in range(0, len(rows), self.sp_batch):
            r = rows[b0:b0 + self.sp_batch]
            if len(r) == r[-1] - r[0] + 1:  # a contiguous run: a view, no gather
                fr, dst = self.frames[int(r[0]):int(r[-1]) + 1], slice(int(r[0]), int(r[-1]) + 1)
            else:
                dst = torch.from_numpy(np.ascontiguousarray(r, np.int64)).to(self.dev)
                fr = self.frames.index_select(0, dst)
            kp, _, ds, _, cnt = self.sp.extract_device(fr)
            if isinstance(dst, slice):
                self.kp_loc[dst].copy_(kp.view(len(r), -1))
                self.ds_loc[dst].copy_(ds.view(len(r), -1))
                self.cnt_loc[dst, 0].copy_(cnt)
            else:
                self.kp_loc.index_copy_(0, dst, kp.view(len(r), -1))
                self.ds_loc.index_copy_(0, dst, ds.view(len(r), -1))
                self.cnt_loc.index_copy_(0, dst, cnt.view(-1, 1).to(self.cnt_loc.dtype))

    def _verify_lightglue(self, pa, pb, dedup, out):
        """SuperPoint features (local table or need-driven exchange) -> LightGlue (once per
        unordered pair when dedup) -> RANSAC + decision + floor gate per ordered pair, for
        this rank's slice (pa, pb) of the pair list (host int32 arrays); fills `out`."""
        self.last_pairs = (pa, pb)
        # features of the keyframes the pairs touch: the local table (world 1), or the
        # need-driven exchange (row k of the compact tables = keyframe need[k])
        if self.world > 1:
            need = np.unique(np.concatenate([pa, pb]).astype(np.int64))
            kp_c, ds_c, cnt_c = self.fx(need, [self.kp_loc, self.ds_loc, self.cnt_loc])
            nf = len(need)
            local = lambda x: np.searchsorted(need, x).astype(np.int32)  # noqa: E731
            out["features_exchanged_bytes"] = self.fx.last_bytes
        else:
            kp_c, ds_c, cnt_c, nf = self.kp_loc, self.ds_loc, self.cnt_loc, self.N
            local = lambda x: np.asarray(x, np.int32)  # noqa: E731
        kp_all = kp_c.view(nf, self.kp, 2)
        ds_all = ds_c.view(nf, self.kp, 256)
        # LightGlue once per UNORDERED pair: it is symmetric in its two images (shared
        # weights; self / cross blocks, dual-softmax assignment, early stopping and pruning
        # treat both alike), so (b, a) is (a, b) with the image roles exchanged and the
        # matches re-sorted by the new image0 index (mlg_lg_orient_matches).  Every ORDERED
        # pair still gets its own RANSAC on its own match order and its own decision, as
        # verify_with_semantics gives each (query, match) (geometric_verification.py:688-744).
        if dedup:
            key = np.minimum(pa, pb).astype(np.int64) * self.N + np.maximum(pa, pb)
            ukey, inv = np.unique(key, return_inverse=True)
            ua, ub = (ukey // self.N).astype(np.int32), (ukey % self.N).astype(np.int32)
            swap_all = (pa > pb).astype(np.uint8)
        else:
            ua, ub, inv, swap_all = pa, pb, np.arange(len(pa)), np.zeros(len(pa), np.uint8)
        order = np.argsort(inv, kind="stable")
        # chunk starts: full chunks, then (lg_tail > 0) the remainder cut so the LAST chunk
        # is 1 / lg_tail of it -- that chunk's RANSAC is the only one with no LightGlue to
        # overlap (per-pair results do not depend on the chunking)
        chunk = self._lg_chunk_for(len(ua))
        self.last_lg_chunk = chunk
        starts = list(range(0, len(ua), chunk))
        rem = len(ua) - starts[-1] if starts else 0
        if self.lg_tail > 0 and rem >= 1024:
            starts.append(len(ua) - max(256, rem // self.lg_tail))
        starts.append(len(ua))
        bounds = np.searchsorted(inv[order], np.asarray(starts))
        out["pairs_matched_lightglue"] = len(ua)
        ua, ub = local(ua), local(ub)  # LightGlue indexes the feature tables
        sp_done = None
        if getattr(self, "_sp_overlap", False):
            # the first chunk's keyframes now, the rest on a side stream under that chunk;
            # only the finished rows' counts are read here (the side stream is
            # writing the others), the rest once the side stream's event has passed
            first = np.unique(np.concatenate([ua[:starts[1]], ub[:starts[1]]])) if len(starts) > 1 else \
                np.zeros(0, np.int64)
            self._extract_rows(first)
            counts = np.zeros(nf, np.int32)
            if len(first):
                fi = self.torch.from_numpy(first.astype(np.int64)).to(self.dev)
                counts[first] = cnt_c.view(-1).index_select(0, fi).cpu().numpy()
            rest = np.setdiff1d(np.arange(self.n_local), first, assume_unique=True)
            sp_done = self._extract_side(rest)
        else:
            counts = cnt_c.view(-1).cpu().numpy()
        # RANSAC of chunk c runs on a side stream while LightGlue matches chunk c + 1 on
        # this one (mlg_lightglue waits on its stream once per layer; the side stream
        # fills those gaps and the CUs the small RANSAC / assignment grids leave idle)
        n_valid_t, gate_rej_t, rec = self._verify_chunks(starts, bounds, order, inv, ua, ub, pa, pb, swap_all, dedup,
                                                         kp_all, ds_all, counts, local, sp_done, cnt_c)
        n_valid, gate_rej = int(n_valid_t), int(gate_rej_t)
        if rec is not None:
            r = {"a": pa, "b": pb, "matches": np.zeros(len(pa), np.int32), "inliers": np.zeros(len(pa), np.int32),
                 "is_valid": np.zeros(len(pa), bool)}
            for sel, n, inl, ok in rec:
                r["matches"][sel] = n.cpu().numpy()
                r["inliers"][sel] = inl.cpu().numpy()
                r["is_valid"][sel] = ok.cpu().numpy()
            self.last_pair_results = r
        out["pairs_verified"] = len(pa)
        out["verified_valid"] = n_valid
        out["verifier_invalid"] = len(pa) - n_valid
        out["gate_rejected_cross_floor"] = gate_rej
        out["accepted"] = n_valid - gate_rej
        return out

    # HBM per LightGlue pair beside its mlg_lightglue workspace: the pair's RANSAC
    # workspace at 1000 hypotheses (models, scores, subsets, points: ~0.9 MB), its flat
    # match coordinates and oriented matches
    _RANSAC_PAIR_BYTES = 1 << 20

    def _lg_chunk_for(self, n_pairs):
        """Pairs per LightGlue call: self.lg_chunk, or with 'auto' the largest multiple of 256
        (<= 5120, bench.py's measured optimum) whose LightGlue + RANSAC workspaces fit in the
        HBM free now (the caching allocator's reusable blocks included), keeping 6 % of the
        device and 4 GiB in reserve."""
        if self.lg_chunk != 'auto':
            return int(self.lg_chunk)
        torch = self.torch
        free, total = torch.cuda.mem_get_info(self.dev)
        free += torch.cuda.memory_reserved(self.dev) - torch.cuda.memory_allocated(self.dev)
        avail = free - 0.06 * total - (4 << 30)
        per = _native.lightglue_workspace_bytes(1024, self.kp) / 1024 + self._RANSAC_PAIR_BYTES
        chunk = int(max(avail, 0) // per) // 256 * 256
        if chunk < 256:
            raise MemoryError(f"LightGlue needs {per * 256 / 2**30:.1f} GiB for 256 pairs; "
                              f"{max(avail, 0) / 2**30:.1f} GiB free")
        return min(chunk, 5120, max(256, -(-n_pairs // 256) * 256))

    def _extract_side(self, rows):
        """_extract_rows on the SuperPoint side stream, after everything already queued on
        the current stream; returns the event the consumers of those rows wait on."""
        torch = self.torch
        main = torch.cuda.current_stream(self.dev)
        if getattr(self, "_sp_stream", None) is None:
            self._sp_stream = torch.cuda.Stream(device=self.dev)
        sps = self._sp_stream
        sps.wait_stream(main)
        with torch.cuda.stream(sps):
            self._extract_rows(rows)
        done = torch.cuda.Event()
        done.record(sps)
        return done

    def _verify_chunks(self, starts, bounds, order, inv, ua, ub, pa, pb, swap_all, dedup, kp_all, ds_all, counts,
                       local, sp_done=None, cnt_c=None):
        torch = self.torch
        from . import geometry
        main = torch.cuda.current_stream(self.dev)
        side = self._side_stream()
        n_valid_t = torch.zeros((), dtype=torch.int64, device=self.dev)
        gate_rej_t = torch.zeros((), dtype=torch.int64, device=self.dev)
        rec = [] if self.record else None
        for ci in range(len(starts) - 1):
            c0, c1 = starts[ci], starts[ci + 1]
            if ci == 1 and sp_done is not None:  # the side-stream SuperPoint rows from here on
                main.wait_event(sp_done)
                counts = cnt_c.view(-1).cpu().numpy()
                sp_done = None
            mu, su, nu, _ = self.lg.match_device(kp_all, ds_all, counts, ua[c0:c1], ub[c0:c1])
            sel = order[bounds[ci]:bounds[ci + 1]]  # the ordered pairs of these unordered ones
            ca, cb = pa[sel], pb[sel]
            if dedup:
                rows = torch.from_numpy((inv[sel] - c0).astype(np.int32)).to(self.dev)
                sw = torch.from_numpy(swap_all[sel]).to(self.dev)
                m, _, n = _native.ops().lg_orient(mu, su, nu, rows, sw)
            else:
                m, n = mu, nu
            ready = torch.cuda.Event()
            ready.record(main)
            with torch.cuda.stream(side):
                side.wait_event(ready)
                m.record_stream(side)
                n.record_stream(side)
                # matched keypoints -> one batched RANSAC (+ recoverPose when K is given).
                # The flat match arrays are laid out on the device without a host sync (no
                # nonzero): pair p's matches go to [offs[p], offs[p] + n[p]) of a buffer of
                # P * kmax rows (RANSAC reads each pair's own range only), the padding of
                # the match lists to one dummy row past the end.
                P = len(ca)
                KP = self.kp
                sidx = torch.arange(KP, device=self.dev)
                lv = sidx[None, :] < n[:, None]
                ta = torch.from_numpy(ca).to(self.dev).long()  # global keyframe indices
                tb = torch.from_numpy(cb).to(self.dev).long()
                la = torch.from_numpy(local(ca)).to(self.dev).long()  # feature-table rows
                lb = torch.from_numpy(local(cb)).to(self.dev).long()
                offs = torch.zeros(P + 1, dtype=torch.int32, device=self.dev)
                offs[1:] = torch.cumsum(n, 0)
                dest = torch.where(lv, offs[:-1, None].long() + sidx[None, :], P * KP).view(-1)
                m0 = torch.where(lv, m[:, :, 0].long(), 0)
                m1 = torch.where(lv, m[:, :, 1].long(), 0)
                k1 = kp_all.new_zeros(P * KP + 1, 2)
                k2 = kp_all.new_zeros(P * KP + 1, 2)
                k1.index_copy_(0, dest, kp_all[la[:, None], m0].view(-1, 2))
                k2.index_copy_(0, dest, kp_all[lb[:, None], m1].view(-1, 2))
                _, _, inl, _, _ = geometry.epipolar_ransac_device(k1[:P * KP], k2[:P * KP], offs, self.K, 0, 3.0)
                ratio = inl.double() / n.clamp(min=1).double()
                ok = (n >= 5) & (inl >= self.min_inliers) & (ratio >= self.min_inlier_ratio)
                n_valid_t += ok.sum()
                if rec is not None:
                    rec.append((sel, n, inl, ok))
                # the floor gate on the geometrically valid pairs.  Deviation, by design: a
                # None label is NaN here and never rejects, where the reference's host gate
                # computes abs(None - None) and raises TypeError (loop_closure_gate.py:89;
                # the drop-in SemanticLoopClosureGate keeps that TypeError,
                # tests/test_api_cpu.py::test_gate_none_labels_raise_nan_labels_accept)
                gate_rej_t += (ok & ((self.f_num[ta] - self.f_num[tb]).abs() > self.limit)).sum()
        if sp_done is not None:  # one chunk only: the tables are complete when step() returns
            main.wait_event(sp_done)
        main.wait_stream(side)
        return n_valid_t, gate_rej_t, rec

    def _verify_loftr(self, pa_t, pb_t, out):
        """verify_with_semantics with GeometricVerifier('loftr') on this rank's slice of the
        pairs (geometric_verification.py:469-526 matches, :104-153 RANSAC, :602-620 rule).
        LoFTR is not symmetric in its images (the fine stage refines in image 1), so every
        ordered pair is matched.  Each rank receives the raw frames its slice touches
        (0.9 MB per keyframe; FeatureExchange over uint8 rows) and runs the backbone on
        them: cheaper to move than the 44 MB of coarse + fine features per keyframe.  Pairs
        go in chunks of loftr_chunk, ordered by (query, match); the backbone features of a
        chunk's keyframes are kept across chunks in a buffer of 2 x 2 x loftr_chunk rows
        and recomputed only for keyframes not already held."""
        torch = self.torch
        from . import geometry
        import time
        if self.time_verify:
            torch.cuda.synchronize(self.dev)
        t_start = time.perf_counter()
        if self.max_pairs is not None:
            pa_t, pb_t = self._first_pairs(pa_t, pb_t, self.max_pairs)
        pa_t, pb_t = self.mdist.balanced_pairs(pa_t, pb_t, self.world, self.rank)
        pa, pb = pa_t.cpu().numpy().astype(np.int64), pb_t.cpu().numpy().astype(np.int64)
        self.last_pairs = (pa, pb)
        need = np.unique(np.concatenate([pa, pb])) if len(pa) else np.zeros(0, np.int64)
        if self.world > 1:
            fl = self.frames.reshape(self.n_local, -1)
            frames = self.fx(need, [fl])[0].view((len(need),) + tuple(self.frames.shape[1:]))
            out["features_exchanged_bytes"] = self.fx.last_bytes
            row_of = {int(f): i for i, f in enumerate(need)}
        else:
            frames = self.frames
            row_of = None
        H, W = int(frames.shape[1]) // 8 * 8, int(frames.shape[2]) // 8 * 8
        order = np.lexsort((pb, pa))
        C = self.loftr_chunk
        cap = 4 * C
        slot_of, free = {}, list(range(cap))
        coarse = fine = None
        n_valid_t = torch.zeros((), dtype=torch.int64, device=self.dev)
        gate_rej_t = torch.zeros((), dtype=torch.int64, device=self.dev)
        rec = [] if self.record else None
        for c0 in range(0, len(order), C):
            sel = order[c0:c0 + C]
            ca, cb = pa[sel], pb[sel]
            frs = np.unique(np.concatenate([ca, cb]))
            keep = set(int(f) for f in frs)
            for f in [f for f in slot_of if f not in keep] if len(free) < len(frs) else []:
                free.append(slot_of.pop(f))
            todo = [int(f) for f in frs if int(f) not in slot_of]
            if todo:
                rows = [f if row_of is None else row_of[f] for f in todo]
                if row_of is None:
                    rows = [f - self.lo for f in rows]
                cf_, ff_ = self.lf.features(frames[torch.as_tensor(rows, device=self.dev)].contiguous())
                if coarse is None:
                    coarse = torch.empty((cap,) + tuple(cf_.shape[1:]), dtype=cf_.dtype, device=self.dev)
                    fine = torch.empty((cap,) + tuple(ff_.shape[1:]), dtype=ff_.dtype, device=self.dev)
                slots = [free.pop() for _ in todo]
                st = torch.as_tensor(slots, device=self.dev)
                coarse.index_copy_(0, st, cf_)
                fine.index_copy_(0, st, ff_)
                slot_of.update(zip(todo, slots))
            n, k0, k1, _ = self.lf.match_device(coarse, fine, H, W, [slot_of[int(a)] for a in ca],
                                                [slot_of[int(b)] for b in cb])
            n = n.to(self.dev).long()
            P = len(sel)
            lv = torch.arange(k0.shape[1], device=self.dev)[None, :] < n[:, None]
            pi, si = torch.nonzero(lv, as_tuple=True)
            offs = torch.zeros(P + 1, dtype=torch.int32, device=self.dev)
            offs[1:] = torch.cumsum(n, 0)
            _, _, inl, _, _ = geometry.epipolar_ransac_device(k0[pi, si].contiguous(), k1[pi, si].contiguous(),
                                                              offs, self.K, 0, 3.0)
            ratio = inl.double() / n.clamp(min=1).double()
            ok = (n >= 5) & (inl >= self.min_inliers) & (ratio >= self.min_inlier_ratio)
            n_valid_t += ok.sum()
            ta = torch.from_numpy(ca).to(self.dev)
            tb = torch.from_numpy(cb).to(self.dev)
            gate_rej_t += (ok & ((self.f_num[ta] - self.f_num[tb]).abs() > self.limit)).sum()
            if rec is not None:
                rec.append((sel, n, inl, ok))
        n_valid, gate_rej = int(n_valid_t), int(gate_rej_t)  # (a device sync)
        if self.time_verify:
            self.last_verify_s = time.perf_counter() - t_start  # this rank's LoFTR verification wall time
        if rec is not None:
            r = {"a": pa, "b": pb, "matches": np.zeros(len(pa), np.int32), "inliers": np.zeros(len(pa), np.int32),
                 "is_valid": np.zeros(len(pa), bool)}
            for sel, n, inl, ok in rec:
                r["matches"][sel] = n.cpu().numpy()
                r["inliers"][sel] = inl.cpu().numpy()
                r["is_valid"][sel] = ok.cpu().numpy()
            self.last_pair_results = r
        out["pairs_verified"] = len(pa)
        out["pairs_matched_loftr"] = len(pa)
        out["verified_valid"] = n_valid
        out["verifier_invalid"] = len(pa) - n_valid
        out["gate_rejected_cross_floor"] = gate_rej
        out["accepted"] = n_valid - gate_rej
        return out

    def _first_pairs(self, pa_t, pb_t, limit):
        """The first `limit` pairs of the global (rank-ordered) pair list, as this rank's part."""
        if self.world == 1:
            return pa_t[:limit], pb_t[:limit]
        torch = self.torch
        n = torch.tensor([pa_t.numel()], dtype=torch.int64, device=self.dev)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        self.mdist.all_gather_into(sizes, n)
        before = sum(int(x.item()) for x in sizes[:self.rank])
        take = max(0, min(pa_t.numel(), limit - before))
        return pa_t[:take], pb_t[:take]

