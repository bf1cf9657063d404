"""Time ocf_encoder_tiles (pre-pass + tile kernel) and the row-gather encoder on one batch of a BASELINE shape,
HIP events around each call, for the library at OCF_LIB_PATH (variants built with -D switches).
    python tools/probes/enc_tiles_probe.py [--config netflix] [--reps 20] [--shards 1]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from omnidirectional_collaborative_filtering_amd import _lib  # noqa: E402
from omnidirectional_collaborative_filtering_amd.data_reader import data_reader  # noqa: E402
from omnidirectional_collaborative_filtering_amd.dataset import synthetic_fixed_split  # noqa: E402
from omnidirectional_collaborative_filtering_amd.engine import cur_stream, ptr  # noqa: E402
from omnidirectional_collaborative_filtering_amd.model import omni_model  # noqa: E402
from omnidirectional_collaborative_filtering_amd.parallel import feature_shard_range  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="netflix")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--shards", type=int, default=1)
ap.add_argument("--tag", default="")
a = ap.parse_args()
data = synthetic_fixed_split(a.config, seed=0)
N, n_rows = data.num_cols, data.train.n_rows
B = 256 * a.shards
shard = None
if a.shards > 1:
    c0, c1 = feature_shard_range(N, 0, a.shards)
    data, shard = data.column_shard(c0, c1), (c0, c1, N)
np.random.seed(1)
rd = data_reader(data.num_cols, n_rows, dataset=data, eval_mode="fixed_split")
om = omni_model(1, 500, data.num_cols, B, dense_activation="sigmoid", use_causal_info=False, compute_dtype="float16",
                seed=3, shard=shard, comm=(lambda t: None) if shard else None)
m = om.model
m.compile("adagrad", "mean_squared_error")
gen = rd.data_gen(B, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
gen._start()
e = om.engine
m._load(None, gen, 1)
out = {"config": a.config, "shards": a.shards, "tag": a.tag, "E": int(e.gt["E"]), "n_tiles": e.n_tiles}
xv = e.gt["xval"]
xv = xv if isinstance(xv, int) else ptr(xv)
g = e._gather_args(e.gt["enc"], 0, e._buf("part_g", e.gt["enc"]["n_chunks"] * e.Hp[0]), e.Hp[0])
g.xval = xv
for name, fn in (("tiles", lambda: e._encoder_tiles("part_enc", e.Hp[0], xv)),
                 ("gather", lambda: _lib.call("ocf_gather_encoder", g, cur_stream()))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(a.reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    out[name + "_us"] = round(ev[0].elapsed_time(ev[1]) * 1e3 / a.reps, 1)
print(json.dumps(out), flush=True)
