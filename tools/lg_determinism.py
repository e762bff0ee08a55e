"""Is LightGlue's output independent of what else runs on the GPU?  (GPU box tool.)

    python tools/lg_determinism.py [--keyframes 5000] [--chunk 2048] [--modes single,threads2,noise]

Builds bench.py's workload once (DeviceGate step: ViT, kNN, SuperPoint), takes the
unordered LightGlue pairs of the step, and matches them chunk by chunk:

  ref       one stream (the product path);
  single    the same again;
  threads2  two host threads, one HIP stream each, alternating chunks (two LightGlue
            calls co-scheduled on the device);
  noise     one stream, while another thread keeps a bf16 GEMM loop busy on a second
            stream (co-scheduling with foreign kernels, no second LightGlue);

and reports, per mode, how many pairs differ from ref in match count, match set
(bitwise) or scores (bitwise).  Run it with tools/ab_run.py --lib-dir for another build.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-level-indoor-slam_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from mlgate import synthetic  # noqa: E402
from mlgate.pipeline import DeviceGate  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402


def run_chunks(gate, kp_all, ds_all, counts, ua, ub, chunk, which, stream, out):
    with torch.cuda.stream(stream):
        for ci in which:
            c0 = ci * chunk
            m, s, n, stop = gate.lg.match_device(kp_all, ds_all, counts, ua[c0:c0 + chunk], ub[c0:c0 + chunk])
            stream.synchronize()
            out[ci] = (m.cpu().numpy(), s.cpu().numpy(), n.cpu().numpy(), stop)


def collect(out, nchunks):
    ms, ss, ns, st = [], [], [], []
    for ci in range(nchunks):
        m, s, n, stop = out[ci]
        ms.append(m)
        ss.append(s)
        ns.append(n)
        st.append(stop)
    return np.concatenate(ms), np.concatenate(ss), np.concatenate(ns), np.concatenate(st)


def compare(ref, got):
    m0, s0, n0, t0 = ref
    m1, s1, n1, t1 = got
    dn = int((n0 != n1).sum())
    dm = ds = 0
    for p in range(len(n0)):
        k = int(n0[p])
        if n0[p] != n1[p] or not np.array_equal(m0[p, :k], m1[p, :k]):
            dm += 1
        elif not np.array_equal(s0[p, :k].view(np.uint32), s1[p, :k].view(np.uint32)):
            ds += 1
    return {"pairs": int(len(n0)), "diff_count": dn, "diff_match_set": dm, "diff_scores_only": ds,
            "diff_stop_layer": int((t0 != t1).sum()), "max_abs_count_diff": int(np.abs(n0 - n1).max())}


def traced(gate, kp_all, ds_all, counts, ua, ub, stream, cap_words=1 << 24):
    """One mlg_lightglue call with the per-stage hash trace on (this thread only):
    (tags, counts, hashes, num_matches)."""
    import ctypes
    from mlgate import _native
    lib = _native.lib()
    buf = torch.zeros(cap_words, dtype=torch.int64, device=kp_all.device)
    _native.check(lib.mlg_dbg_lg_trace_begin(_native.ptr(buf), cap_words * 8), "trace_begin")
    with torch.cuda.stream(stream):
        m, s, n, stop = gate.lg.match_device(kp_all, ds_all, counts, ua, ub)
    stream.synchronize()
    tags = np.zeros(8192, np.int32)
    cnts = np.zeros(8192, np.int32)
    k = lib.mlg_dbg_lg_trace_end(tags.ctypes.data_as(ctypes.c_void_p), cnts.ctypes.data_as(ctypes.c_void_p), 8192)
    if k < 0:
        raise RuntimeError(f"trace buffer too small ({k})")
    used = int(cnts[:k].sum())
    return tags[:k], cnts[:k], buf[:used].cpu().numpy(), n.cpu().numpy()


def first_divergence(ref, got):
    t0, c0, h0, n0 = ref
    t1, c1, h1, n1 = got
    out = {"stages": int(len(t0)), "stages_got": int(len(t1)), "diff_count": int((n0 != n1).sum())}
    o = 0
    for i in range(min(len(t0), len(t1))):
        if t0[i] != t1[i] or c0[i] != c1[i]:
            out["first"] = {"stage_index": i, "tag_ref": int(t0[i]), "tag_got": int(t1[i]), "layout_differs": True}
            return out
        a, b = h0[o:o + c0[i]], h1[o:o + c0[i]]
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0]
            out["first"] = {"stage_index": i, "tag": int(t0[i]), "tiles": int(c0[i]), "tiles_differing": int(len(bad)),
                            "first_tiles": bad[:8].tolist(),
                            "previous_tags": [int(x) for x in t0[max(0, i - 4):i]]}
            return out
        o += c0[i]
    out["first"] = None
    return out


def differing_tags(ref, got, limit=16):
    t0, c0, h0, _ = ref
    t1, c1, h1, _ = got
    if len(t0) != len(t1) or not np.array_equal(t0, t1) or not np.array_equal(c0, c1):
        return ["layout differs"]
    o, tags = 0, []
    for i in range(len(t0)):
        if not np.array_equal(h0[o:o + c0[i]], h1[o:o + c0[i]]):
            tags.append(int(t0[i]))
        o += c0[i]
    return tags[:limit]


def trace_mode(gate, kp_all, ds_all, counts, ua, ub, chunk, nch, dev, pairs, repeats):
    """Trace the first `pairs` pairs alone, then again while a second thread runs the
    other chunks on its own stream; name the first stage whose hashes differ."""
    s0 = torch.cuda.current_stream(dev)
    ta, tb = ua[:pairs], ub[:pairs]
    ref = traced(gate, kp_all, ds_all, counts, ta, tb, s0)
    again = traced(gate, kp_all, ds_all, counts, ta, tb, s0)
    res = {"alone_again": first_divergence(ref, again)}
    res["alone_again"]["differing_tags"] = differing_tags(ref, again)
    for r in range(repeats):
        st = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        box = {}
        other = threading.Thread(target=run_chunks, args=(gate, kp_all, ds_all, counts, ua, ub, chunk,
                                                          list(range(1, min(nch, 3))), st[1], {}))
        other.start()
        time.sleep(0.05)
        box["got"] = traced(gate, kp_all, ds_all, counts, ta, tb, st[0])
        other.join()
        res[f"with_second_call_{r}"] = first_divergence(ref, box["got"])
        res[f"with_second_call_{r}"]["differing_tags"] = differing_tags(ref, box["got"])
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keyframes", type=int, default=5000)
    ap.add_argument("--chunk", type=int, default=1024)
    ap.add_argument("--modes", default="single,threads2,noise")
    ap.add_argument("--max-pairs", type=int, default=0)
    ap.add_argument("--trace-pairs", type=int, default=512)
    ap.add_argument("--trace-repeats", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    seq, labels = bench.sequence(a.keyframes, 600)
    frames = synthetic.frames_device(seq, np.arange(a.keyframes), dev)
    gate = DeviceGate(frames, seq.t, labels, 1, 0, dev, k=20, verify=True, K=bench.ISEC_K, vit_batch=123, sp_batch=64,
                      lg_chunk=a.chunk, vit_state_dict=synthetic_state_dict(0))
    t0 = time.time()
    gate.step()
    torch.cuda.synchronize()
    pa, pb = gate.last_pairs
    key = np.unique(np.minimum(pa, pb).astype(np.int64) * gate.N + np.maximum(pa, pb))
    ua, ub = (key // gate.N).astype(np.int32), (key % gate.N).astype(np.int32)
    if a.max_pairs:
        ua, ub = ua[:a.max_pairs], ub[:a.max_pairs]
    kp_all = gate.kp_loc.view(gate.N, gate.kp, 2)
    ds_all = gate.ds_loc.view(gate.N, gate.kp, 256)
    counts = gate.cnt_loc.view(-1).cpu().numpy()
    nch = (len(ua) + a.chunk - 1) // a.chunk
    print(json.dumps({"setup_s": round(time.time() - t0, 1), "unordered_pairs": int(len(ua)), "chunks": nch}),
          flush=True)
    main_stream = torch.cuda.current_stream(dev)

    def single():
        out = {}
        run_chunks(gate, kp_all, ds_all, counts, ua, ub, a.chunk, range(nch), main_stream, out)
        return collect(out, nch)

    modes = a.modes.split(",")
    res = {}
    if "trace" in modes:
        t = time.time()
        res["trace"] = trace_mode(gate, kp_all, ds_all, counts, ua, ub, a.chunk, nch, dev, a.trace_pairs,
                                  a.trace_repeats)
        res["trace"]["seconds"] = round(time.time() - t, 2)
        print(json.dumps({"trace": res["trace"]}), flush=True)
        modes = [m for m in modes if m != "trace"]
        torch.cuda.empty_cache()
    ref = single() if modes else None
    for mode in modes:
        t = time.time()
        torch.cuda.empty_cache()
        if mode == "single":
            got = single()
        elif mode == "threads2":
            out = {}
            streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
            th = [threading.Thread(target=run_chunks, args=(gate, kp_all, ds_all, counts, ua, ub, a.chunk,
                                                             range(i, nch, 2), streams[i], out)) for i in range(2)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            got = collect(out, nch)
        elif mode == "noise":
            stop = threading.Event()
            ns = torch.cuda.Stream(dev)
            A = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)

            def noise():
                with torch.cuda.stream(ns):
                    while not stop.is_set():
                        for _ in range(8):
                            torch.matmul(A, A)
                        ns.synchronize()
            nt = threading.Thread(target=noise)
            nt.start()
            try:
                got = single()
            finally:
                stop.set()
                nt.join()
        else:
            raise SystemExit(f"unknown mode {mode}")
        res[mode] = compare(ref, got)
        res[mode]["seconds"] = round(time.time() - t, 2)
        print(json.dumps({mode: res[mode]}), flush=True)
    print(json.dumps({"summary": res}), flush=True)


if __name__ == "__main__":
    main()
