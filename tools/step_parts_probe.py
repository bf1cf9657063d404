"""Where a small config's GPU step goes (GPU box): the one-call step's four launches timed one at a time
from its verified template (ocf_train_step_rows' members), and each weight-gradient launch without its
folded jobs / without rows, to separate the jobs' dependent-load chains from the row stream.  Timing only:
the launches repeat on the same batch (the weights drift; nothing is checked).
    python tools/step_parts_probe.py [config] [dtype]"""
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from omnidirectional_collaborative_filtering_amd import _lib, optimizers as O  # noqa: E402
from omnidirectional_collaborative_filtering_amd.data_reader import data_reader  # noqa: E402
from omnidirectional_collaborative_filtering_amd.dataset import synthetic_fixed_split  # noqa: E402
from omnidirectional_collaborative_filtering_amd.engine import cur_stream  # noqa: E402
from omnidirectional_collaborative_filtering_amd.model import omni_model  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "ml1m"
cd = sys.argv[2] if len(sys.argv) > 2 else "bfloat16"
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
for i in range(6):
    eng.fast_train_step(gen, i % gen.num_batches)
torch.cuda.synchronize()
st = eng._plan["st"]
s = cur_stream()
L = _lib.load()


def timed(fn, n=60):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / n * 1e3, 2)


def gemm(g):
    return lambda: _lib.call("ocf_gemm", g, s)


cp = lambda g: type(g).from_buffer_copy(g)
out = cp(st.dw_out)
out.jr = ctypes.addressof(st.jr) if st.jr_on else None
res = {"enc": timed(lambda: _lib.call("ocf_gather_encoder", st.enc, s)),
       "dec": timed(lambda: _lib.call("ocf_gather_decoder", st.dec, s)),
       "dw_out": timed(gemm(out)), "dw_in": timed(gemm(st.dw_in)),
       "step": timed(lambda: _lib.call("ocf_train_step_rows", st, s), 40)}
o2 = cp(out)
o2.jr = None
res["dw_out_no_jr"] = timed(gemm(o2))
o3 = cp(o2)
o3.cb_p = o3.cb_s1 = o3.cb_s2 = None
res["dw_out_no_jobs"] = timed(gemm(o3))
i2 = cp(st.dw_in)
i2.jb_part = None
res["dw_in_no_bias_job"] = timed(gemm(i2))
i3 = cp(i2)
i3.js_sp = None
res["dw_in_no_jobs"] = timed(gemm(i3))
# rows only over an empty live list: the launch + jobs floor (records of zero rows)
z = torch.zeros_like(torch.as_tensor(np.zeros(1)))
live0 = torch.zeros(eng.Np // 128 * _lib.LIVE_REC, dtype=torch.uint8, device="cuda")
i4 = cp(i3)
i4.row_live = live0.data_ptr()
res["dw_in_no_jobs_no_rows"] = timed(gemm(i4))
i5 = cp(st.dw_in)
i5.row_live = live0.data_ptr()
res["dw_in_jobs_only"] = timed(gemm(i5))
o4 = cp(out)
o4.row_live = live0.data_ptr()
res["dw_out_jobs_only"] = timed(gemm(o4))
print(json.dumps(dict(config=cfg, dtype=cd, us=res)))
# the pair launch (ocf_gemm_pair): without the row reduction (nothing to wait for) and with it (the engine's
# running counter: nothing to clear between launches)
sync = ctypes.addressof(eng.pair_state)
res["pair_no_jr"] = timed(lambda: _lib.call("ocf_gemm_pair", o2, st.dw_in, sync, s))
res["pair_jr"] = timed(lambda: _lib.call("ocf_gemm_pair", out, st.dw_in, sync, s))
res["two_launches_jr"] = timed(lambda: (_lib.call("ocf_gemm", out, s), _lib.call("ocf_gemm", st.dw_in, s)))
print(json.dumps(dict(config=cfg, dtype=cd, pair=res)))
