"""LiDAR floor tracking: drop-in mirror of scripts/semantic_gating/lidar_floor_tracker.py
(LiDARFloorTracker, MultiModalFloorDetector, FloorEstimate).

The per-scan compute -- ground-candidate extraction and the ground-plane RANSAC
(lidar_floor_tracker.py:70-141) -- runs on the GPU, for any number of scans at once
(``process_scans``): ring / height masks on the device, then ``mlg_plane_ransac``
(one launch for all scans).  The tracker's sequential state (z history, reference
height, floor numbers, transitions, label lookup) is a few scalars per scan and stays
on the host, with the reference's exact arithmetic.

The reference samples its RANSAC hypotheses from numpy's unseeded global RNG; here
they come from a seeded counter-based stream, so plane, ratio and floor decisions are
deterministic.
"""
from collections import deque
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import _native
from .floors import IMUFloorDetector


@dataclass
class FloorEstimate:
    """Single floor estimate from LiDAR"""
    timestamp: float
    z_height: float
    floor_number: int
    confidence: float
    num_ground_points: int


def ground_plane_ransac_device(pts, offs, iterations, threshold, seed=0):
    """pts device f32 [N, 3], offs device int32 [S + 1] -> device (plane f64 [S, 4], ratio f64 [S],
    inliers int32 [S])."""
    plane, ratio, inl = _native.ops().plane_ransac(pts.contiguous(), offs.contiguous(), int(iterations),
                                                   int(seed) & ((1 << 63) - 1), float(threshold))
    return plane, ratio, inl


class LiDARFloorTracker:
    """Track robot height from LiDAR ground plane detection (RANSAC on the GPU).

    Same constructor as the reference; ``device`` ('cuda') and ``seed`` (0, the RANSAC
    sampling stream) are attributes a caller may set after construction."""

    device = 'cuda'
    seed = 0

    def __init__(self, floor_height: float = 3.5, ground_ring_threshold: int = 30, ransac_iterations: int = 100,
                 ransac_threshold: float = 0.1, min_ground_points: int = 100, smoothing_window: int = 10):
        self.floor_height = floor_height
        self.ground_ring_threshold = ground_ring_threshold
        self.ransac_iterations = ransac_iterations
        self.ransac_threshold = ransac_threshold
        self.min_ground_points = min_ground_points
        self.smoothing_window = smoothing_window
        self.z_history: deque = deque(maxlen=smoothing_window)
        self.floor_history: List[FloorEstimate] = []
        self.current_floor: int = 0
        self.reference_z: Optional[float] = None

    # ------------------------------------------------------------ GPU stages
    def _ground_device(self, pts, rings):
        """Ground candidates of one scan on the device (lidar_floor_tracker.py:70-90)."""
        if rings is not None:
            return pts[rings < self.ground_ring_threshold]
        z = pts[:, 2]
        # np.percentile(z, 5) with linear interpolation, from two order statistics
        n = z.numel()
        pos = 0.05 * (n - 1)
        lo = int(np.floor(pos))
        frac = pos - lo
        srt_lo = torch.kthvalue(z, lo + 1).values
        srt_hi = torch.kthvalue(z, min(lo + 2, n)).values if frac > 0 else srt_lo
        z_min = srt_lo + (srt_hi - srt_lo) * frac
        return pts[z < (z_min + 0.5)]

    def extract_ground_points(self, points: np.ndarray, rings: Optional[np.ndarray] = None) -> np.ndarray:
        dev = _native.require_device(self.device)
        p = torch.as_tensor(np.ascontiguousarray(points, np.float32)).to(dev)
        r = None if rings is None else torch.as_tensor(np.asarray(rings)).to(dev)
        return self._ground_device(p, r).cpu().numpy()

    def fit_ground_plane_ransac(self, points: np.ndarray) -> Tuple[Optional[np.ndarray], float]:
        if len(points) < 3:
            return None, 0.0
        plane, ratio, _ = self._ransac([np.asarray(points, np.float32)])
        return plane[0], ratio[0]

    def _ransac(self, ground_list):
        dev = _native.require_device(self.device)
        sizes = [len(g) for g in ground_list]
        offs = np.zeros(len(sizes) + 1, np.int32)
        np.cumsum(sizes, out=offs[1:])
        pts = torch.cat([g if torch.is_tensor(g) else torch.as_tensor(np.ascontiguousarray(g, np.float32)).to(dev)
                         for g in ground_list]).reshape(-1, 3).float().contiguous()
        plane, ratio, _ = ground_plane_ransac_device(pts, torch.from_numpy(offs).to(dev), self.ransac_iterations,
                                                     self.ransac_threshold, self.seed)
        plane, ratio = plane.cpu().numpy(), ratio.cpu().numpy()
        planes = [None if (n < 3 or np.isnan(pl[0])) else pl for pl, n in zip(plane, sizes)]
        return planes, [float(r) if n >= 3 else 0.0 for r, n in zip(ratio, sizes)]

    # ------------------------------------------------------------ host state
    def estimate_robot_height(self, plane_params: np.ndarray) -> float:
        a, b, c, d = plane_params
        height = abs(d)
        if c < 0:
            height = -height
        return height

    def _update(self, timestamp, n_ground, plane, ratio) -> FloorEstimate:
        if n_ground < self.min_ground_points or plane is None:
            return FloorEstimate(timestamp=timestamp, z_height=self.z_history[-1] if self.z_history else 0.0,
                                 floor_number=self.current_floor, confidence=0.0, num_ground_points=n_ground)
        z_height = self.estimate_robot_height(plane)
        self.z_history.append(z_height)
        if self.reference_z is None:
            self.reference_z = z_height
        smoothed_z = np.mean(self.z_history)
        floor_number = int(round((smoothed_z - self.reference_z) / self.floor_height))
        z_variance = np.var(self.z_history) if len(self.z_history) > 1 else 1.0
        confidence = ratio * (1.0 / (1.0 + z_variance * 10))
        self.current_floor = floor_number
        est = FloorEstimate(timestamp=timestamp, z_height=smoothed_z, floor_number=floor_number,
                            confidence=confidence, num_ground_points=n_ground)
        self.floor_history.append(est)
        return est

    def process_scan(self, points: np.ndarray, timestamp: float, rings: Optional[np.ndarray] = None) -> FloorEstimate:
        return self.process_scans([points], [timestamp], None if rings is None else [rings])[0]

    def process_scans(self, points_list, timestamps, rings_list=None) -> List[FloorEstimate]:
        """Batched process_scan: ground extraction + RANSAC for every scan in one GPU pass,
        then the tracker's state update in scan order (identical to calling process_scan
        per scan)."""
        dev = _native.require_device(self.device)
        grounds = []
        for i, pts in enumerate(points_list):
            p = torch.as_tensor(np.ascontiguousarray(pts, np.float32)).to(dev)
            r = None if rings_list is None or rings_list[i] is None else torch.as_tensor(np.asarray(rings_list[i])).to(dev)
            grounds.append(self._ground_device(p, r))
        n_ground = [int(g.shape[0]) for g in grounds]
        run = [i for i, n in enumerate(n_ground) if n >= self.min_ground_points]
        planes, ratios = ([], []) if not run else self._ransac([grounds[i] for i in run])
        fit = {i: (planes[j], ratios[j]) for j, i in enumerate(run)}
        return [self._update(t, n_ground[i], *fit.get(i, (None, 0.0))) for i, t in enumerate(timestamps)]

    def detect_floor_transitions(self, min_duration: float = 2.0) -> List[Tuple[float, int, int]]:
        if len(self.floor_history) < 2:
            return []
        transitions = []
        last_floor = self.floor_history[0].floor_number
        last_time = self.floor_history[0].timestamp
        for est in self.floor_history[1:]:
            if est.floor_number != last_floor:
                if est.timestamp - last_time >= min_duration:
                    transitions.append((est.timestamp, last_floor, est.floor_number))
                    last_time = est.timestamp
                last_floor = est.floor_number
        return transitions

    def get_floor_labels(self, timestamps: np.ndarray) -> np.ndarray:
        if len(self.floor_history) == 0:
            return np.zeros(len(timestamps), dtype=int)
        scan_times = np.array([e.timestamp for e in self.floor_history])
        scan_floors = np.array([e.floor_number for e in self.floor_history])
        idx = np.argmin(np.abs(scan_times[None, :] - np.asarray(timestamps)[:, None]), axis=1)
        return scan_floors[idx].astype(int)

    def reset(self):
        self.z_history.clear()
        self.floor_history.clear()
        self.current_floor = 0
        self.reference_z = None


class MultiModalFloorDetector:
    """IMU transitions + LiDAR height (lidar_floor_tracker.py:309-404); the fusion keeps
    the IMU labels, as the reference does."""

    def __init__(self, floor_height: float = 3.5, imu_weight: float = 0.7, lidar_weight: float = 0.3):
        self.floor_height = floor_height
        self.imu_weight = imu_weight
        self.lidar_weight = lidar_weight
        self.imu_detector = IMUFloorDetector()
        self.lidar_tracker = LiDARFloorTracker(floor_height=floor_height)
        self.fused_floor_labels: Optional[np.ndarray] = None

    def process_imu(self, timestamps, accel_x, accel_y, accel_z):
        self.imu_detector.detect_elevator_events(timestamps, accel_x, accel_y, accel_z)

    def process_lidar_scan(self, points: np.ndarray, timestamp: float, rings: Optional[np.ndarray] = None):
        self.lidar_tracker.process_scan(points, timestamp, rings)

    def fuse_estimates(self, trajectory_times: np.ndarray, start_floor: int = 0) -> np.ndarray:
        imu_labels = self.imu_detector.assign_floor_labels(trajectory_times, start_floor)
        if len(self.lidar_tracker.floor_history) > 0:
            lidar_labels = self.lidar_tracker.get_floor_labels(trajectory_times)
            lidar_labels = lidar_labels + (start_floor - lidar_labels[0])  # noqa: F841 (reference keeps IMU)
        self.fused_floor_labels = imu_labels.copy()
        return self.fused_floor_labels

    def get_floor_at_time(self, t: float) -> int:
        if self.fused_floor_labels is None:
            raise ValueError("Call fuse_estimates first")
        raise NotImplementedError("Use fuse_estimates result directly")
