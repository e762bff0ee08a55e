"""Bench-scale verifier decisions against the fp32 chain.

tests/golden/decision_sample.npz: a seeded uniform sample (seed 2026, no margin filter)
of 600 of the 32,568 ordered pairs one bench step verifies (5000 keyframes, 600 places,
k = 20), with
  * the GPU full gate's per-pair LightGlue match count, RANSAC inlier count and decision
    (tools/decision_sample.py, DeviceGate(record=True) on host-generated keyframes);
  * the fp32 chain's (tools/decision_check_cpu.py, this container: oracle.pipeline
    .verify_pair -- SuperPoint and LightGlue without bf16 emulation, OpenCV's RANSAC loop
    restated, the decision rule of geometric_verification.py:602-620).
The fixture holds 0 decision flips in 600 (214 valid both ways).

GPU test: the sampled pairs re-verified through the drop-in GeometricVerifier
(verify_frames_batch: SuperPoint per keyframe, one ragged LightGlue call, batched RANSAC)
give the fp32 chain's decision on every pair, and match / inlier counts within the bf16
chain's spread of the fixture (median relative match-count difference <= 2 %, 99th
percentile <= 15 %, inliers of valid pairs within 10 %).  The fixture's own GPU columns
(the kernels of its generation) are kept for reference; a kernel change that moves
rounding is expected to move counts slightly, never the decisions."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_sampled_bench_pairs_reproduce_and_match_fp32_decisions(dev, golden_dir):
    import bench
    from mlgate import synthetic
    from mlgate.verify import GeometricVerifier
    d = np.load(f"{golden_dir}/decision_sample.npz")
    assert int(np.sum(d["is_valid"] != d["fp32_is_valid"])) == 0
    seq, _ = bench.sequence(int(d["keyframes"]), int(d["places"]))
    used = np.unique(np.concatenate([d["a"], d["b"]]))
    pos = {int(f): i for i, f in enumerate(used)}
    frames = torch.empty(len(used), synthetic.H, synthetic.W, 3, dtype=torch.uint8, device=dev)
    for b0 in range(0, len(used), 128):
        frames[b0:b0 + 128].copy_(torch.from_numpy(synthetic.frames_host(seq, used[b0:b0 + 128])))
    v = GeometricVerifier('lightglue', device=str(dev))
    pairs = [(pos[int(a)], pos[int(b)]) for a, b in zip(d["a"], d["b"])]
    res = v.verify_frames_batch(frames, pairs, bench.ISEC_K)
    got_m = np.array([r.num_matches for r in res])
    got_i = np.array([r.num_inliers for r in res])
    got_v = np.array([r.is_valid for r in res])
    assert np.array_equal(got_v, d["fp32_is_valid"]), np.flatnonzero(got_v != d["fp32_is_valid"])[:10]
    fm, fi = d["fp32_matches"].astype(np.float64), d["fp32_inliers"].astype(np.float64)
    rel_m = np.abs(got_m - fm) / np.maximum(fm, 1.0)
    assert np.median(rel_m) <= 0.02 and np.quantile(rel_m, 0.99) <= 0.15, (np.median(rel_m), np.quantile(rel_m, 0.99))
    v = d["fp32_is_valid"]
    rel_i = np.abs(got_i[v] - fi[v]) / np.maximum(fi[v], 1.0)
    assert rel_i.max() <= 0.10, rel_i.max()
