"""Diagnostic: LightGlue run-to-run and batched-vs-single score differences."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-level-indoor-slam_amd"), os.path.join(ROOT, "tests")]
from test_lightglue_gpu import feats, _run_gpu  # noqa: E402
from mlgate.lightglue import LightGlueGPU  # noqa: E402
from mlgate.weights import lightglue_state_dict  # noqa: E402

kw = dict(depth_confidence=-1, width_confidence=-1) if os.environ.get("NOPRUNE") else {}
lg = LightGlueGPU(lightglue_state_dict(0), device="cuda", **kw)
rng = np.random.default_rng(3)
cases = [feats(rng, 300, 280), feats(rng, 1600, 1550), feats(rng, 40, 90), feats(rng, 800, 10)]
b1 = _run_gpu(lg, cases)
b2 = _run_gpu(lg, cases)
for i, c in enumerate(cases):
    s1 = _run_gpu(lg, [c])[0]
    s2 = _run_gpu(lg, [c])[0]
    def d(a, b):
        return (len(a[0]), len(b[0]), float(np.abs(a[1] - b[1]).max()) if len(a[1]) == len(b[1]) and len(a[1]) else -1)
    print(i, "single-single", d(s1, s2), "batch-batch", d(b1[i], b2[i]), "single-batch", d(s1, b1[i]), s1[2], b1[i][2])
