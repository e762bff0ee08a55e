"""The full gate at SURVEY §8d's stress size on one GPU: N = 19,163
keyframes, the ORB-SLAM3 pose count of the reference's ISEC run
(orb_slam3_integration.py:167-217 gates that trajectory), through DeviceGate exactly as
bench.py runs N = 5000 -- split-bf16 ViT, fused kNN gate (k = 20), SuperPoint 2048,
LightGlue, OpenCV-sequenced E-RANSAC, the decision rule and the floor gate -- with the
LightGlue chunk sized from the free HBM (lg_chunk='auto') and the local-feature cache
unmaterialised (the gate never reads it; 31 GB at this N).

Checks: retrieval rows sampled across the sequence equal the oracle's per-row loop
(oracle/csrc/oracle.c, find_loop_closures :851-911) on the same similarity rows; the
four rejection terms and the pair counts are self-consistent; every ordered pair's
decision is the reference rule on its own (matches, inliers)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N = 19163


def test_full_gate_at_orbslam3_pose_count(dev):
    import bench
    from mlgate import retrieval, synthetic
    from mlgate.pipeline import DeviceGate
    from mlgate.weights import synthetic_state_dict
    from oracle import _lib
    seq, labels = bench.sequence(N, 2300)  # bench.py's 600 places per 5000 keyframes, scaled
    frames = synthetic.frames_device(seq, np.arange(N), dev)
    gate = DeviceGate(frames, seq.t, labels, 1, 0, dev, k=20, verify=True, K=bench.ISEC_K, vit_batch=246,
                      lg_chunk="auto", local_features=False, vit_state_dict=synthetic_state_dict(0), record=True)
    out = gate.step()
    torch.cuda.synchronize()
    assert gate.local_feats is None and 256 <= gate.last_lg_chunk <= 5120
    idx, sim, valid, count = gate.last_retrieval
    # (1) retrieval: sampled rows against the oracle's loop on the same f32 similarity rows
    X = gate.gather.out
    rows = np.arange(0, N, 491)
    S = retrieval.similarity(X[torch.from_numpy(rows).to(dev)], X).cpu().numpy()
    codes, has = gate.h_codes, gate.h_has
    for j, r in enumerate(rows):
        oi, osim, ov, oc = _lib.knn_rows(S[j:j + 1], int(r), seq.t, codes, has, 10.0, 0.5, 20, True)
        c = count[r]
        assert c == oc[0] and np.array_equal(idx[r, :c], oi[0, :c]) and np.array_equal(sim[r, :c], osim[0, :c]), r
        assert np.array_equal(valid[r, :c].astype(bool), ov[0, :c].astype(bool)), r
    # (2) the counts: every emitted match is floor-rejected, skipped or verified; every
    # verified pair is valid or invalid; accepted = valid - cross-floor rejections
    live = np.arange(idx.shape[1])[None, :] < count[:, None]
    assert out["matches"] == int(count.sum())
    assert out["retrieval_floor_rejected"] == int((live & (valid == 0)).sum())
    assert out["pairs_verified"] == out["matches"] - out["retrieval_floor_rejected"] - out["skipped_floor_mismatch"]
    assert out["verified_valid"] + out["verifier_invalid"] == out["pairs_verified"]
    assert out["accepted"] == out["verified_valid"] - out["gate_rejected_cross_floor"]
    assert out["pairs_verified"] > 4 * 32000 * 0.8 and out["verified_valid"] > 0
    # (3) every decision is the rule on that pair's own counts (geometric_verification.py:602-620)
    r = gate.last_pair_results
    n, inl = r["matches"].astype(np.int64), r["inliers"].astype(np.int64)
    rule = (n >= 5) & (inl >= 20) & (inl / np.maximum(n, 1) >= 0.25)
    assert len(n) == out["pairs_verified"] and np.array_equal(r["is_valid"], rule)
    assert int(r["is_valid"].sum()) == out["verified_valid"]
    print({k: v for k, v in out.items()}, "lg_chunk", gate.last_lg_chunk)
