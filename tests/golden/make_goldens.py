"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run ONLY in the build container, where the reference is mounted read-only at
/root/reference (it never travels to the GPU box; only the .npz/.json vectors
written here do):

    python tests/golden/make_goldens.py

Every fixture is data: seeded inputs plus what the reference's own public API
returned for them.  Inputs are constructed so that nothing depends on the
reference's unstable sort (np.argsort default kind) or on a borderline float
comparison: every similarity that decides a top-k boundary or the threshold test is
kept >= MARGIN away from its neighbour / the threshold (checked below, the seed is
re-rolled otherwise).

What is captured (reference file:line in parentheses):
  knn_*.npz        SemanticPlaceRecognition.find_loop_closures + get_statistics
                   (place_recognition.py:851-933) on injected PlaceDescriptors
  pairwise.npz     BasePlaceRecognition.compute_all_pairwise_similarities (:179-190)
  query.npz        BasePlaceRecognition.query (:117-163) with the extractor stubbed
  xcorr.npz        CricaVPR.compute_cross_correlation_score / rerank_candidates (:669-757)
  gate.json        SemanticLoopClosureGate demo + random candidates, strict and not
                   (loop_closure_gate.py:60-134, demo :261-304)
  imu.npz          IMUFloorDetector.detect_elevator_events / assign_floor_labels
                   (floor_detector.py:63-156)
  verifier.json    SemanticGeometricVerifier cross-floor skip branch + stats
                   (geometric_verification.py:688-744)
  traj_*.npz       trajectory-proximity candidates + floor gate counts of the
                   ORB-SLAM3 / LeGO-LOAM integrations (orb_slam3_integration.py:167-281,
                   lego_loam_integration.py:121-204) with the positions they used
"""
import hashlib
import json
import os
import sys
import warnings

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
MARGIN = 1e-5  # > 2x the float32 summation-order tolerance of the parity tests (4e-6)


def _import_reference():
    if not os.path.isdir(REF):
        raise SystemExit("reference not mounted; goldens can only be regenerated in the build container")
    sys.path.insert(0, REF)
    warnings.simplefilter("ignore")
    import scripts.semantic_gating as sg  # noqa: E402
    return sg


def clustered_descriptors(rng, n, d, n_places, spread):
    """Revisited places: each keyframe = its place centre + isotropic noise."""
    centres = rng.standard_normal((n_places, d)).astype(np.float32)
    place = rng.integers(0, n_places, n)
    scale = rng.uniform(0.4 * spread, 1.6 * spread, (n, 1)).astype(np.float32)  # varied revisit quality
    noise = rng.standard_normal((n, d)).astype(np.float32) * scale
    # values on the float16 grid so the fixture can store them losslessly as float16
    return (centres[place] + noise).astype(np.float16).astype(np.float32), place


def margins_ok(sim, t, min_gap, k, thr):
    """True when no decision of find_loop_closures sits within MARGIN of a flip."""
    n = sim.shape[0]
    for i in range(n):
        s = sim[i].astype(np.float64).copy()
        s[np.abs(t - t[i]) < min_gap] = -np.inf
        v = np.sort(s[np.isfinite(s)])[::-1]
        if v.size == 0:
            continue
        if np.min(np.abs(v[:k] - thr)) < MARGIN:
            return False
        # only the order of emitted entries (>= thr) and the k-th/(k+1)-th boundary
        # while the k-th is still emitted can change the reference's output
        above = int(np.sum(v[:k] >= thr))
        top = v[: min(above + 1, k + 1, v.size)]
        if above > 0 and top.size > 1 and np.min(np.abs(np.diff(top))) < MARGIN:
            return False
    return True


def knn_case(sg, name, seed, n, d, k, thr, gap, gating, none_frac, n_places, spread, dt=0.765):
    from scripts.semantic_gating.place_recognition import PlaceDescriptor, SemanticPlaceRecognition
    for attempt in range(400):
        rng = np.random.default_rng(seed + 1000 * attempt)
        X, place = clustered_descriptors(rng, n, d, n_places, spread)
        t = np.arange(n, dtype=np.float64) * dt + rng.uniform(0, 0.01, n)
        blocks = np.array([5, 1, 4, 2])
        floor = blocks[np.minimum((np.arange(n) * 4) // max(n, 1), 3)]
        # perceptual aliasing: some places appear on another floor too
        alias = rng.random(n) < 0.25
        floor = np.where(alias, blocks[rng.integers(0, 4, n)], floor).astype(np.int64)
        has_floor = rng.random(n) >= none_frac
        Xn = X / (np.linalg.norm(X, axis=1, keepdims=True) + 1e-8)
        if margins_ok(Xn @ Xn.T, t, gap, k, thr):
            break
    else:
        raise RuntimeError(f"could not build a tie-free case for {name}")
    spr = SemanticPlaceRecognition("mixvpr", device="cpu", similarity_threshold=thr, min_time_gap=gap)
    for i in range(n):
        spr.vpr.descriptors.append(PlaceDescriptor(
            timestamp=float(t[i]), descriptor=X[i],
            floor_label=int(floor[i]) if has_floor[i] else None))
    matches = spr.find_loop_closures(enable_floor_gating=gating, k=k)
    stats = spr.get_statistics(matches)
    np.savez_compressed(
        os.path.join(OUT, f"knn_{name}.npz"),
        desc=X.astype(np.float16), t=t, floor=floor, has_floor=has_floor.astype(np.uint8),
        params=np.array([k, thr, gap, int(gating)], dtype=np.float64),
        q=np.array([m.query_idx for m in matches], np.int64),
        m=np.array([m.match_idx for m in matches], np.int64),
        sim=np.array([m.similarity for m in matches], np.float64),
        qt=np.array([m.query_timestamp for m in matches], np.float64),
        mt=np.array([m.match_timestamp for m in matches], np.float64),
        valid=np.array([m.is_valid for m in matches], np.uint8),
        stats=json.dumps({kk: float(vv) for kk, vv in stats.items()}),
    )
    return len(matches)


def pairwise_case(sg):
    from scripts.semantic_gating.place_recognition import PlaceDescriptor, CricaVPR
    rng = np.random.default_rng(7)
    X, _ = clustered_descriptors(rng, 96, 768, 20, 0.7)
    vpr = CricaVPR(device="cpu")
    for i in range(96):
        vpr.descriptors.append(PlaceDescriptor(timestamp=float(i), descriptor=X[i]))
    S = vpr.compute_all_pairwise_similarities()
    M = vpr.build_descriptor_matrix()
    empty = CricaVPR(device="cpu").compute_all_pairwise_similarities()
    np.savez_compressed(os.path.join(OUT, "pairwise.npz"), desc=X.astype(np.float16), S=S, M=M, empty_size=np.int64(empty.size))


def query_case(sg):
    from scripts.semantic_gating.place_recognition import PlaceDescriptor, MixVPR
    rng = np.random.default_rng(11)
    X, _ = clustered_descriptors(rng, 200, 4096, 30, 0.6)
    qd = (X[17] + rng.standard_normal(4096).astype(np.float32) * np.float32(0.3)).astype(np.float16).astype(np.float32)
    t = np.arange(200, dtype=np.float64) * 0.765
    vpr = MixVPR(device="cpu")
    vpr.extract_descriptor = lambda image: qd.astype(np.float32)
    for i in range(200):
        vpr.descriptors.append(PlaceDescriptor(timestamp=float(t[i]), descriptor=X[i]))
    out = {}
    for tag, ts, k, gap in (("a", 20.0, 5, 10.0), ("b", None, 5, 10.0), ("c", 100.0, 12, 30.0)):
        ms = vpr.query(None, timestamp=ts, k=k, min_time_gap=gap)
        out[f"{tag}_m"] = np.array([m.match_idx for m in ms], np.int64)
        out[f"{tag}_sim"] = np.array([m.similarity for m in ms], np.float64)
        out[f"{tag}_q"] = np.array([m.query_idx for m in ms], np.int64)
    np.savez_compressed(os.path.join(OUT, "query.npz"), desc=X.astype(np.float16), t=t, qdesc=qd, **out)


def xcorr_case(sg):
    from scripts.semantic_gating.place_recognition import CricaVPR
    import torch
    torch.set_num_threads(4)
    rng = np.random.default_rng(5)
    feats = rng.standard_normal((6, 1, 528, 768)).astype(np.float32)
    feats[1] = feats[0] + 0.5 * rng.standard_normal((1, 528, 768)).astype(np.float32)
    feats[2] = feats[0][:, rng.permutation(528)] + 0.3 * rng.standard_normal((1, 528, 768)).astype(np.float32)
    feats = feats.astype(np.float16).astype(np.float32)
    vpr = CricaVPR(device="cpu", use_reranking=True)
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (4, 5), (3, 3)]
    scores = np.array([vpr.compute_cross_correlation_score(feats[a], feats[b]) for a, b in pairs], np.float64)
    # 2-D inputs (no batch dim) take the same path after squeeze
    s2d = vpr.compute_cross_correlation_score(feats[0][0], feats[1][0])
    for i in range(5):
        vpr._feature_cache[i] = feats[i]
    cands = [(1, 0.61), (2, 0.72), (3, 0.93), (5, 0.55), (4, 0.40)]
    rr = vpr.rerank_candidates(0, cands, top_k=4)
    rr_nocache = vpr.rerank_candidates(5, cands, top_k=3)
    np.savez_compressed(
        os.path.join(OUT, "xcorr.npz"), feats=feats.astype(np.float16), pairs=np.array(pairs, np.int64), scores=scores,
        s2d=np.float64(s2d), cands=np.array(cands, np.float64),
        rr=np.array(rr, np.float64), rr_nocache=np.array(rr_nocache, np.float64))


def gate_case(sg):
    from scripts.semantic_gating.loop_closure_gate import SemanticLoopClosureGate
    labels = np.zeros(10000, dtype=int)
    labels[0:5000] = 5
    labels[5000:7000] = 1
    labels[7000:8500] = 4
    labels[8500:10000] = 2
    demo = [(100, 4500, 0.85), (200, 5500, 0.92), (5100, 6800, 0.88), (300, 7200, 0.91),
            (7100, 8200, 0.87), (400, 9000, 0.93), (4000, 4200, 0.80)]
    rng = np.random.default_rng(3)
    rnd = [(int(a), int(b), float(s)) for a, b, s in
           zip(rng.integers(0, 10000, 5000), rng.integers(0, 10000, 5000), rng.random(5000))]
    out = {"labels_blocks": [[0, 5000, 5], [5000, 7000, 1], [7000, 8500, 4], [8500, 10000, 2]]}
    for strict in (True, False):
        for tag, cands in (("demo", demo), ("random", rnd)):
            g = SemanticLoopClosureGate(labels, strict_mode=strict)
            valid, rejected = g.gate_candidates(cands)
            key = f"{tag}_{'strict' if strict else 'loose'}"
            out[key] = {
                "candidates": cands,
                "valid": [[c.query_idx, c.match_idx, float(c.similarity_score), int(c.query_floor),
                           int(c.match_floor)] for c in valid],
                "rejected": [[c.query_idx, c.match_idx, c.rejection_reason] for c in rejected],
                "stats": {k: float(v) for k, v in g.get_stats().items()},
            }
    g = SemanticLoopClosureGate(labels)
    out["empty_stats"] = {k: float(v) for k, v in g.get_stats().items()}
    with open(os.path.join(OUT, "gate.json"), "w") as f:
        json.dump(out, f)


def imu_case(sg):
    from scripts.semantic_gating.floor_detector import IMUFloorDetector
    rng = np.random.default_rng(21)
    dt = 1 / 200
    t = np.arange(0, 240, dt)
    n = len(t)
    ax = rng.normal(0, 0.1, n)
    ay = rng.normal(0, 0.1, n)
    az = rng.normal(9.81, 0.1, n)
    rides = [(20.0, 25.0, 0.8), (70.0, 74.5, -0.7), (130.0, 131.0, 0.9), (160.0, 166.0, 0.75),
             (238.0, 240.0, 0.8)]  # short ride rejected; last ride still open at the end
    for a, b, g in rides:
        az[(t >= a) & (t <= b)] += g
    ax[(t >= 200) & (t <= 205)] += rng.normal(0, 2.0, ((t >= 200) & (t <= 205)).sum())
    az[(t >= 200) & (t <= 205)] += 0.8  # high horizontal variance: not an elevator
    det = IMUFloorDetector()
    ev = det.detect_elevator_events(t, ax, ay, az)
    traj = np.linspace(0, 240, 3000)
    labels = det.assign_floor_labels(traj, start_floor=5)
    evarr = np.array([[e.start_time, e.end_time, e.duration, e.start_idx, e.end_idx, e.floor_change]
                      for e in ev], np.float64).reshape(-1, 6)
    np.savez_compressed(os.path.join(OUT, "imu.npz"), t=t, ax=ax, ay=ay, az=az, traj=traj,
                        events=evarr, directions=np.array([e.direction for e in ev]), labels=labels)


def verifier_case(sg):
    from scripts.semantic_gating.geometric_verification import SemanticGeometricVerifier, MatchResult
    v = SemanticGeometricVerifier(device="cpu")
    res = [v.verify_with_semantics(None, None, f1, f2, None, q, m)
           for (f1, f2, q, m) in ((1, 2, 3, 4), (5, 1, 7, 9), (2, 4, 0, 0))]
    out = {"results": [{k: (None if val is None else val) for k, val in r.__dict__.items()} for r in res],
           "stats": v.get_statistics(), "fresh_stats": SemanticGeometricVerifier(device="cpu").get_statistics(),
           "fields": list(MatchResult.__dataclass_fields__.keys())}
    with open(os.path.join(OUT, "verifier.json"), "w") as f:
        json.dump(out, f)


def traj_case(sg, system):
    from scripts.semantic_gating import orb_slam3_integration as orb, lego_loam_integration as lego
    cls = {"orb_slam3": orb.ORBSlam3SemanticIntegration, "lego_loam": lego.LegoLoamSemanticIntegration}[system]
    import io, contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        integ = cls(trajectory_dir=f"{REF}/results/trajectories/{system}", **(
            {"dataset_dir": "/nonexistent"} if system == "orb_slam3" else {}), output_dir="/tmp/mlgate_goldens_out")
        integ.load_trajectories()
        integ.combine_trajectories()
        cands = integ.detect_loop_closure_candidates()
        analysis = integ.apply_floor_gating(cands)
    pos = integ.combined_trajectory[:, 1:4].astype(np.float64)
    ij = np.array([(a, b) for a, b, _ in cands], np.int64)
    n = len(pos)
    key = np.sort(ij[:, 0] * n + ij[:, 1])
    digest = hashlib.sha256(key.astype("<i8").tobytes()).hexdigest()
    np.savez_compressed(
        os.path.join(OUT, f"traj_{system}.npz"), pos=pos, floor=integ.floor_labels.astype(np.int64),
        total=np.int64(analysis.total_candidates), same=np.int64(analysis.same_floor_candidates),
        cross=np.int64(analysis.cross_floor_candidates),
        first_cross=np.array([p[:2] for p in analysis.cross_floor_pairs[:5]], np.int64),
        gate_stats=json.dumps({k: float(v) for k, v in integ.loop_gate.get_stats().items()}),
        pair_sha256=digest, pair_key_sum=np.uint64(int(key.sum()) % (1 << 64)))
    return analysis.total_candidates


def _params(fn):
    import inspect
    return [[p.name, None if p.default is inspect.Parameter.empty else repr(p.default)]
            for p in inspect.signature(fn).parameters.values()]


def api_case(sg):
    """Public signatures / dataclass fields of the reference API (the drop-in contract)."""
    import dataclasses
    import inspect
    from scripts.semantic_gating import floor_detector, geometric_verification, lidar_floor_tracker, loop_closure_gate
    from scripts.semantic_gating import place_recognition
    out = {}
    for mod in (floor_detector, loop_closure_gate, place_recognition, geometric_verification, lidar_floor_tracker):
        for name, obj in vars(mod).items():
            if name.startswith('_') or getattr(obj, '__module__', None) != mod.__name__:
                continue
            if inspect.isclass(obj):
                entry = {}
                if dataclasses.is_dataclass(obj):
                    entry['__fields__'] = [(f.name, repr(f.default) if f.default is not dataclasses.MISSING
                                            else None) for f in dataclasses.fields(obj)]
                for mname, m in vars(obj).items():
                    if inspect.isfunction(m) and (not mname.startswith('_') or mname == '__init__'):
                        entry[mname] = _params(m)
                out[name] = entry
            elif inspect.isfunction(obj):
                out[name] = _params(obj)
    out['__all__'] = list(sg.__all__)
    with open(os.path.join(OUT, "api.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def snippet_case(sg):
    """integrate_with_orbslam3's return value (a C++ snippet string) -- loop_closure_gate.py:223-257."""
    from scripts.semantic_gating import loop_closure_gate
    out = {"integrate_with_orbslam3": loop_closure_gate.integrate_with_orbslam3(np.array([1, 1, 2]),
                                                                                np.array([0.0, 1.0, 2.0]))}
    with open(os.path.join(OUT, "gate_snippet.json"), "w") as f:
        json.dump(out, f, indent=1)


def main():
    sg = _import_reference()
    api_case(sg)
    snippet_case(sg)
    if "--api-only" in sys.argv:
        return
    print("reference", sg.__version__)
    print("knn small", knn_case(sg, "small", 1, 64, 768, 10, 0.5, 10.0, True, 0.0, 8, 0.6))
    print("knn gaps", knn_case(sg, "gaps", 2, 300, 768, 10, 0.5, 10.0, True, 0.1, 40, 0.8))
    print("knn nogate", knn_case(sg, "nogate", 3, 300, 768, 7, 0.6, 5.0, False, 0.0, 40, 0.8))
    print("knn k20", knn_case(sg, "k20", 4, 500, 768, 20, 0.45, 10.0, True, 0.0, 30, 0.9))
    print("knn d4096", knn_case(sg, "d4096", 5, 200, 4096, 10, 0.5, 10.0, True, 0.05, 25, 0.9))
    print("knn wide", knn_case(sg, "wide", 6, 2000, 768, 6, 0.55, 10.0, True, 0.0, 400, 1.0))
    print("knn selfgap0", knn_case(sg, "selfgap0", 8, 120, 768, 5, 0.5, 0.0, True, 0.0, 20, 0.8))
    print("knn tiny", knn_case(sg, "tiny", 9, 3, 768, 10, -1.0, 0.5, True, 0.0, 1, 0.5))
    pairwise_case(sg)
    query_case(sg)
    xcorr_case(sg)
    gate_case(sg)
    imu_case(sg)
    verifier_case(sg)
    print("traj lego", traj_case(sg, "lego_loam"))
    print("traj orb", traj_case(sg, "orb_slam3"))


if __name__ == "__main__":
    main()
