"""Per-phase timing of the fused small-model step (ocf_mlp_step) on the Jester configuration: workgroup 0's
100 MHz clock at the start and at every grid barrier (arrive / leave), averaged over steps.
    python tools/mlp_trace.py [--dtype bfloat16] [--wgs 0]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import jester_arrays  # noqa: E402
from omnidirectional_collaborative_filtering_amd.model import omni_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dtype", default="bfloat16")
ap.add_argument("--wgs", type=int, default=0)
ap.add_argument("--steps", type=int, default=30)
a = ap.parse_args()


def trace_of(e):
    t = e.mlp_trace.cpu().numpy().astype(np.float64)
    n = int(np.count_nonzero(t))
    return np.diff(t[:n]) / 100.0                  # us between marks


inputs, observed, out_m, targets = jester_arrays(n=20000)
om = omni_model(2, 256, 100, 128, dense_activation="tanh", use_causal_info=True, compute_dtype=a.dtype, seed=3)
m = om.model
m.compile("rmsprop", "mean_squared_error")
e = om.engine
e.mlp_trace = torch.zeros(24, dtype=torch.int64, device="cuda")
e.mlp_wgs = a.wgs
xd = [torch.as_tensor(z).cuda() for z in (inputs, observed, out_m)]
yd = torch.as_tensor(targets).cuda()
idx = torch.arange(20000, device="cuda")
rows = []
for s in range(a.steps):
    m._load_rows(xd, yd, idx[s * 128:(s + 1) * 128])
    e.train_step()
    torch.cuda.synchronize()
    t = e.mlp_trace.cpu().numpy().astype(np.float64)
    n = int(np.count_nonzero(t))
    rows.append(np.diff(t[:n]) / 100.0)          # us between marks
d = np.mean(rows[3:], axis=0)
print(json.dumps({"dtype": a.dtype, "wgs": a.wgs or "default", "us_between_marks": [round(x, 2) for x in d],
                  "total_us": round(float(d.sum()), 2),
                  "marks": "start, then per barrier: arrive, leave; last: end"}))
