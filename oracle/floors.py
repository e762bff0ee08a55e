"""Oracle for IMU floor labelling (test infrastructure only).

Restates IMUFloorDetector.detect_elevator_events / assign_floor_labels
(floor_detector.py:63-156): median detrend of a_z, scipy uniform_filter1d
(mode='reflect') smoothing, mask |a_z| > thr & smoothed horizontal energy < thr_h,
segments closed only on a falling edge (a ride still open at the end of the log is
dropped), duration >= min, direction from the sign of the trapezoid integral;
labels: poses in [last_end, start) get the current floor, poses inside a ride keep 0.
"""
import numpy as np
from scipy.ndimage import uniform_filter1d


def detect_events(t, ax, ay, az, z_thr=0.5, min_duration=2.0, window=50, h_thr=1.0):
    az_s = uniform_filter1d(az - np.median(az), size=window)
    hv = uniform_filter1d(ax ** 2 + ay ** 2, size=window)
    mask = (np.abs(az_s) > z_thr) & (hv < h_thr)
    m = mask.astype(np.int8)
    edges = np.diff(np.concatenate(([0], m)))
    starts = np.flatnonzero(edges == 1)
    ends = np.flatnonzero(edges == -1)  # falling edge at index i (mask[i] False)
    events = []
    for s in starts:
        e = ends[ends > s]
        if e.size == 0:
            continue
        e = int(e[0])
        dur = t[e] - t[s]
        if dur >= min_duration:
            seg = az_s[s:e]
            ts = t[s:e]
            integ = np.sum((ts[1:] - ts[:-1]) * (seg[1:] + seg[:-1]) / 2.0)
            up = integ > 0
            events.append((t[s], t[e], dur, 'up' if up else 'down', int(s), e, 1 if up else -1))
    return events


def assign_labels(traj_t, events, start_floor=5):
    traj_t = np.asarray(traj_t)
    labels = np.zeros(len(traj_t), dtype=int)
    cur = start_floor
    last_end = traj_t[0]
    for ev in sorted(events, key=lambda e: e[0]):
        labels[(traj_t >= last_end) & (traj_t < ev[0])] = cur
        cur += ev[6]
        last_end = ev[1]
    labels[traj_t >= last_end] = cur
    return labels
