"""Seeded synthetic multi-floor keyframe sequences (the bench / test workload).

There is no ISEC data and no network, so the workload is generated.  It follows the
reference's own synthetic scenes (geometric_verification.py:752-774: filled rectangles
on black plus U[0, 30) noise) and the ISEC sequence shape:

  * a *place* is a seeded rectangle scene; keyframe i shows place ``place_of[i]``,
    shifted by (sx, sy) in {-8, 0, 8} px (one SuperPoint cell: the untrained
    synthetic networks are exactly shift-equivariant at that stride, so a revisit
    yields true correspondences) plus fresh noise;
  * places recur on several floors (perceptual aliasing the floor gate must stop);
  * t_i = i * 0.765 s (the DROID keyframe spacing, droid_slam_semantic_analysis.txt:7-9);
  * floors follow a plan of (floor, fraction) blocks -- ISEC's 5 / 1 / 4 / 2 with
    45.5 / 13.3 / 13.6 / 27.6 % by default (semantic_gating_comparison.txt:29-33);
  * a 200 Hz IMU log realises every floor change as |df| elevator rides of
    +-0.8 m/s^2 (floor_detector.py:207-223 style), so IMUFloorDetector recovers the
    labels (keyframes inside a ride get label 0, as the reference assigns them, and
    show the elevator car -- one shared scene).
"""
from dataclasses import dataclass

import numpy as np

H, W = 480, 640
SHIFTS = (-8, 0, 8)
KF_DT = 0.765
ISEC_PLAN = ((5, 0.455), (1, 0.133), (4, 0.136), (2, 0.276))
RIDE_S, PAUSE_S, IMU_HZ = 4.0, 3.0, 200.0


def scene(seed, h=H, w=W):
    """A place: 20-40 filled rectangles (colours 60-255) on black, uint8 [h, w, 3] BGR."""
    r = np.random.default_rng(1000 + int(seed))
    img = np.zeros((h, w, 3), np.uint8)
    for _ in range(int(r.integers(20, 40))):
        x, y = int(r.integers(0, w - 60)), int(r.integers(0, h - 60))
        ww, hh = int(r.integers(20, 120)), int(r.integers(20, 120))
        img[y:y + hh, x:x + ww] = r.integers(60, 255, 3)
    return img


@dataclass
class Sequence:
    place_of: np.ndarray   # int [N]
    shift: np.ndarray      # int [N, 2] (sx, sy)
    t: np.ndarray          # float64 [N] keyframe timestamps
    floor_gt: np.ndarray   # int [N] floor the keyframe was taken on (0 inside a ride)
    rides: list            # [(t_start, t_end, +1 / -1)]
    seed: int

    @property
    def n(self):
        return len(self.t)


def make_sequence(n, places, seed=0, plan=ISEC_PLAN):
    """Keyframe i at t_i = i * 0.765 s.  Floors change between plan blocks by |df|
    consecutive elevator rides (RIDE_S long, PAUSE_S apart); keyframes taken during a
    ride see the elevator car (place -1) and carry floor 0."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) * KF_DT
    cuts = np.round(np.cumsum([f for _, f in plan]) * n).astype(int)
    rides = []
    t_free = -np.inf  # rides of one transition follow each other; a transition never
    for b in range(1, len(plan)):  # starts before the previous one has finished
        i0 = min(int(cuts[b - 1]), n - 1)
        df = plan[b][0] - plan[b - 1][0]
        t0 = max(t[i0] - 0.5 * KF_DT, t_free)  # rides start between keyframes
        for _ in range(abs(df)):
            rides.append((t0, t0 + RIDE_S, 1 if df > 0 else -1))
            t0 += RIDE_S + PAUSE_S
        t_free = t0
    place_of = rng.integers(0, places, size=n)
    shift = rng.choice(np.array(SHIFTS), size=(n, 2))
    floor_gt = np.full(n, plan[0][0], np.int64)
    cur = plan[0][0]
    for (a, b, d) in rides:
        inside = (t >= a) & (t < b)
        cur += d
        floor_gt[t >= b] = cur
        floor_gt[inside] = 0
        place_of[inside] = -1
    return Sequence(place_of=place_of, shift=shift, t=t, floor_gt=floor_gt, rides=rides, seed=seed)


ELEVATOR_SCENE = 999_983  # the elevator car's interior is one more (shared) place


def _base(place, h, w):
    return scene(ELEVATOR_SCENE if place < 0 else place, h, w)


def frames_host(seq, idx=None, h=H, w=W):
    """uint8 [len(idx), h, w, 3] keyframes (numpy noise; test-sized batches)."""
    idx = np.arange(seq.n) if idx is None else np.asarray(idx)
    out = np.empty((len(idx), h, w, 3), np.uint8)
    cache = {}
    for j, i in enumerate(idx):
        p = int(seq.place_of[i])
        if p not in cache:
            cache[p] = _base(p, h, w)
        sx, sy = (int(v) for v in seq.shift[i])
        noise = np.random.default_rng((seq.seed + 1) * 1_000_003 + int(i)).integers(0, 30, (h, w, 3))
        out[j] = np.clip(np.roll(cache[p], (sy, sx), (0, 1)).astype(np.int16) + noise, 0, 255)
    return out


def frames_device(seq, idx, device, h=H, w=W):
    """Same scenes generated on the device (torch noise; for bench-sized sequences, where
    host generation of 5000 x 921,600 B would dominate start-up).  Keyframe i's noise is
    draw i of one seeded Philox stream whichever frames are rendered: the generator offset
    is set per frame (i x one draw's increment), so a rank's shard arange(lo, hi) equals
    rows lo..hi of the whole sequence bit for bit (the sharded bench gates the single-rank
    bench's frames)."""
    import torch
    idx = np.asarray(idx)
    g = torch.Generator(device=device).manual_seed(seq.seed)
    base = g.get_offset()
    probe = torch.Generator(device=device).manual_seed(seq.seed)
    torch.randint(0, 30, (h, w, 3), generator=probe, device=device, dtype=torch.int16)
    inc = probe.get_offset() - base
    out = torch.empty(len(idx), h, w, 3, dtype=torch.uint8, device=device)
    bases = {}
    for j, i in enumerate(idx):
        p = int(seq.place_of[i])
        if p not in bases:
            bases[p] = torch.from_numpy(_base(p, h, w)).to(device)
        sx, sy = (int(v) for v in seq.shift[i])
        g.set_offset(base + int(i) * inc)
        fr = torch.roll(bases[p], shifts=(sy, sx), dims=(0, 1)).to(torch.int16)
        fr = fr + torch.randint(0, 30, fr.shape, generator=g, device=device, dtype=torch.int16)
        out[j] = fr.clamp_(0, 255).to(torch.uint8)
    return out


def imu_log(seq, rate=IMU_HZ, seed=None):
    """(t, ax, ay, az) at `rate` Hz covering the sequence: gravity + N(0, 0.1) noise, and
    +-0.8 m/s^2 on a_z during each ride (floor_detector.py:207-223)."""
    rng = np.random.default_rng(seq.seed + 7 if seed is None else seed)
    t = np.arange(0.0, seq.t[-1] + 2.0, 1.0 / rate)
    n = len(t)
    ax = rng.normal(0, 0.1, n)
    ay = rng.normal(0, 0.1, n)
    az = rng.normal(9.81, 0.1, n)
    for a, b, d in seq.rides:
        az[(t >= a) & (t <= b)] += 0.8 * d
    return t, ax, ay, az
