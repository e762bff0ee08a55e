"""IMU floor labelling: drop-in mirror of scripts/semantic_gating/floor_detector.py.

Produces the per-keyframe floor labels the gate consumes (BASELINE configs[3]).  It
is host-side work by design (a 200 Hz IMU log is kilobytes), so it
runs vectorised in numpy/scipy: segment detection by edge finding instead of a
per-sample Python loop, identical decisions (falling-edge closure, ride still open at
the end of the log dropped, duration >= min, trapezoid-integral direction) and
identical labels (poses inside a ride keep label 0).
"""
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np
from scipy.ndimage import uniform_filter1d


@dataclass
class ElevatorEvent:
    """A detected elevator ride."""
    start_time: float
    end_time: float
    duration: float
    direction: str
    start_idx: int
    end_idx: int
    floor_change: int


class IMUFloorDetector:
    """Elevator rides from sustained vertical acceleration with little horizontal motion."""

    def __init__(self, z_accel_threshold: float = 0.5, min_duration: float = 2.0, window_size: int = 50,
                 horizontal_var_threshold: float = 1.0):
        self.z_accel_threshold = z_accel_threshold
        self.min_duration = min_duration
        self.window_size = window_size
        self.horizontal_var_threshold = horizontal_var_threshold
        self.events: List[ElevatorEvent] = []
        self.floor_labels: Optional[np.ndarray] = None

    def detect_elevator_events(self, timestamps: np.ndarray, accel_x: np.ndarray, accel_y: np.ndarray,
                               accel_z: np.ndarray) -> List[ElevatorEvent]:
        az = uniform_filter1d(accel_z - np.median(accel_z), size=self.window_size)
        horiz = uniform_filter1d(accel_x ** 2 + accel_y ** 2, size=self.window_size)
        on = (np.abs(az) > self.z_accel_threshold) & (horiz < self.horizontal_var_threshold)
        step = np.diff(on.astype(np.int8), prepend=np.int8(0))
        rises = np.flatnonzero(step == 1)
        falls = np.flatnonzero(step == -1)
        self.events = []
        for s in rises:
            after = falls[falls > s]
            if after.size == 0:  # still inside a ride when the log ends: never closed
                break
            e = int(after[0])
            dur = timestamps[e] - timestamps[s]
            if dur >= self.min_duration:
                seg, ts = az[s:e], timestamps[s:e]
                area = np.sum(np.diff(ts) * (seg[1:] + seg[:-1]) / 2.0)
                up = area > 0
                self.events.append(ElevatorEvent(start_time=timestamps[s], end_time=timestamps[e], duration=dur,
                                                 direction='up' if up else 'down', start_idx=int(s), end_idx=e,
                                                 floor_change=1 if up else -1))
        return self.events

    def assign_floor_labels(self, trajectory_times: np.ndarray, start_floor: int = 5) -> np.ndarray:
        tt = np.asarray(trajectory_times)
        labels = np.zeros(len(tt), dtype=int)
        floor, since = start_floor, tt[0]
        for ev in sorted(self.events, key=lambda e: e.start_time):
            labels[(tt >= since) & (tt < ev.start_time)] = floor
            floor += ev.floor_change
            since = ev.end_time
        labels[tt >= since] = floor
        self.floor_labels = labels
        return labels

    def get_floor_at_time(self, t: float) -> int:
        if self.floor_labels is None:
            raise ValueError("Call assign_floor_labels first")
        raise NotImplementedError("Use assign_floor_labels result directly")


def load_imu_from_bag(bag_path: str, imu_topic: str = '/vectornav/imu') -> Tuple[np.ndarray, ...]:
    """(t, ax, ay, az, gx, gy, gz) arrays from a ROS1 bag (needs the ROS `rosbag` module)."""
    try:
        import rosbag
    except ImportError as e:
        raise ImportError("rosbag not available. Run inside ROS environment.") from e
    cols = [[] for _ in range(7)]
    with rosbag.Bag(bag_path, 'r') as bag:
        for _, msg, t in bag.read_messages(topics=[imu_topic]):
            la, av = msg.linear_acceleration, msg.angular_velocity
            for c, v in zip(cols, (t.to_sec(), la.x, la.y, la.z, av.x, av.y, av.z)):
                c.append(v)
    return tuple(np.array(c) for c in cols)
