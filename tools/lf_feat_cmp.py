"""Compare two tools/lf_feat_dump.py outputs: per array max |d|, differing elements and the
first differing (frame, pixel) positions (A/B diagnostics)."""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for k in ("coarse", "fine"):
    d = np.abs(a[k] - b[k])
    print(k, a[k].shape, "max", float(d.max()), "differing", int((d > 0).sum()), "of", d.size)
    if (d > 0).any():
        idx = np.argwhere(d > 0)
        px = np.unique(idx[:, 1])
        print("  pixels differing", len(px), "first", px[:12].tolist(), "frames", np.unique(idx[:, 0]).tolist())
        i = tuple(idx[0])
        print("  e.g.", i, float(a[k][i]), float(b[k][i]))
