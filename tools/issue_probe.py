"""Host cost of issuing a training step (GPU box): the general path (Python argument blocks, four library
calls), the one-call step (Engine.fast_train_step), ocf_train_step_rows alone, and a one-kernel library call.
Each is timed over bursts short enough for the GPU queue to absorb them (host time only), then synchronised.
    python tools/issue_probe.py [config] [dtype]"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from omnidirectional_collaborative_filtering_amd import _lib, optimizers as O  # noqa: E402
from omnidirectional_collaborative_filtering_amd.data_reader import data_reader  # noqa: E402
from omnidirectional_collaborative_filtering_amd.dataset import synthetic_fixed_split  # noqa: E402
from omnidirectional_collaborative_filtering_amd.engine import cur_stream  # noqa: E402
from omnidirectional_collaborative_filtering_amd.model import omni_model  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "ml100k"
cd = sys.argv[2] if len(sys.argv) > 2 else "float32"
data = synthetic_fixed_split(cfg, seed=0)
np.random.seed(1234)
rd = data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split", rng="numpy")
om = omni_model(1, 500, data.num_cols, 256, dense_activation="sigmoid", use_causal_info=False,
                dropout_probability=0.2, compute_dtype=cd, seed=7)
m = om.model
m.compile(O.Adagrad(lr=0.005, epsilon=1e-8), "mean_squared_error")
eng = om.engine
gen = rd.data_gen(256, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
gen._start()
nb = gen.num_batches
for i in range(6):
    eng.fast_train_step(gen, i % nb)
torch.cuda.synchronize()
assert eng._plan.get("ready")
res = {}


def burst(name, fn, n=40, reps=20):
    ts = []
    for r in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(n):
            fn(i)
        ts.append((time.perf_counter() - t) / n * 1e6)
        torch.cuda.synchronize()
    res[name] = round(float(np.median(ts)), 2)


burst("fast_train_step_us", lambda i: eng.fast_train_step(gen, i % nb))
st = eng._plan["st"]
s = cur_stream()
burst("ocf_train_step_rows_call_us", lambda i: _lib.call("ocf_train_step_rows", st, s))
x = torch.zeros(256 * 512, device="cuda")
y = torch.zeros(512, device="cuda")
burst("one_kernel_call_us", lambda i: _lib.call("ocf_colsum", x.data_ptr(), 0, 512, 4, 512, 1.0, y.data_ptr(), s))
burst("general_path_us", lambda i: (m._load(None, gen, i % nb), eng.train_step()))
t = time.perf_counter()
for i in range(400):
    eng.fast_train_step(gen, i % nb)
torch.cuda.synchronize()
res["fast_steady_ms_per_step"] = round((time.perf_counter() - t) / 400 * 1e3, 4)
t = time.perf_counter()
for i in range(400):
    m._load(None, gen, i % nb)
    eng.train_step()
torch.cuda.synchronize()
res["general_steady_ms_per_step"] = round((time.perf_counter() - t) / 400 * 1e3, 4)
print(json.dumps(dict(config=cfg, dtype=cd, **res)))
