"""ViT descriptor determinism probe: batch composition, run-to-run and two concurrent
streams, bitwise (diagnostic for tests/test_distributed_gpu.py)."""
import json
import sys
import threading

import numpy as np
import torch

sys.path.insert(0, "multi-level-indoor-slam_amd")
from mlgate import synthetic  # noqa: E402
from mlgate.vit import VitB14  # noqa: E402
from mlgate.weights import synthetic_state_dict  # noqa: E402

dev = torch.device("cuda:0")
seq = synthetic.make_sequence(300, 60, 3)
fr = torch.from_numpy(synthetic.frames_host(seq, np.arange(300))).to(dev)
sd = synthetic_state_dict(0)
res = {}


def run(batch, x=fr, stream=None):
    eng = VitB14(sd, device="cuda", max_batch=batch, precise=False)
    if stream is None:
        d = eng.forward(x)
    else:
        with torch.cuda.stream(stream):
            d = eng.forward(x)
    torch.cuda.synchronize()
    return d.cpu()


ref = run(123)
for b in (123, 50, 1):
    d = run(b) if b != 1 else torch.cat([run(1, fr[i:i + 1]) for i in range(40)])
    n = d.shape[0]
    res[f"batch{b}"] = {"rows_differ": int((d != ref[:n]).any(1).sum()), "max_abs": float((d - ref[:n]).abs().max())}
# shifted position: frames 5.. in a batch starting at 5
d = run(123, fr[5:])
res["shift5"] = {"rows_differ": int((d != ref[5:]).any(1).sum()), "max_abs": float((d - ref[5:]).abs().max())}
# two concurrent streams
outs = [None, None]
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def th(i, s):
    outs[i] = run(123, fr, s)


ts = [threading.Thread(target=th, args=(i, s)) for i, s in enumerate((s1, s2))]
[t.start() for t in ts]
[t.join() for t in ts]
for i in range(2):
    res[f"concurrent{i}"] = {"rows_differ": int((outs[i] != ref).any(1).sum()),
                             "max_abs": float((outs[i] - ref).abs().max())}
print(json.dumps(res))
