"""Where the ML-20M encoder/decoder launch goes (GPU box): the one-call step's gather members timed one at a time
from its verified template -- the fused launch, the encoder alone, the decoder alone with and without its row
reduction -- with the W-row bytes each reads.  Timing only: the launches repeat on the same batch.
    python tools/probes/encdec_probe.py [config] [dtype]"""
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

cfg = sys.argv[1] if len(sys.argv) > 1 else "ml20m"
cd = sys.argv[2] if len(sys.argv) > 2 else "float16"
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
    eng.fast_train_step(gen, 3)
torch.cuda.synchronize()
st = eng._plan["st"]
s = cur_stream()


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


cp = lambda g: type(g).from_buffer_copy(g)
dec = cp(st.dec)
dec.jr = ctypes.addressof(st.jr) if st.jr_on == 2 else None
E = int(gen.nnz1[3])
wrow = eng.Hp[0] * (2 if cd != "float32" else 4)
res = {"entries": E, "w_row_bytes": wrow, "enc_chunks": st.enc.n_chunks, "dec_chunks": dec.n_chunks,
       "fused_in_template": bool(st.enc_arrive)}
if st.enc_arrive:
    res["fused"] = timed(lambda: _lib.call("ocf_gather_encdec", st.enc, dec, st.enc_arrive, s))
    prev = ctypes.c_int32()
    _lib.call("ocf_set_tuning", b"encdec_rowres", 1, ctypes.byref(prev))
    res["fused_rowres"] = timed(lambda: _lib.call("ocf_gather_encdec", st.enc, dec, st.enc_arrive, s))
    _lib.call("ocf_set_tuning", b"encdec_rowres", prev.value, None)
res["enc"] = timed(lambda: _lib.call("ocf_gather_encoder", st.enc, s))
res["dec_with_reduction"] = timed(lambda: _lib.call("ocf_gather_decoder", dec, s))
d2 = cp(dec)
d2.jr = None
d2.row_arrive = None
res["dec_no_reduction"] = timed(lambda: _lib.call("ocf_gather_decoder", d2, s))
d3 = cp(d2)
d3.enc_part = None          # h read from the stored activations instead of the encoder partials' epilogue
res["dec_no_reduction_no_epilogue"] = timed(lambda: _lib.call("ocf_gather_decoder", d3, s))
for k in ("fused", "fused_rowres", "enc", "dec_with_reduction", "dec_no_reduction", "dec_no_reduction_no_epilogue"):
    if k in res:
        n = 2 if k.startswith("fused") else 1
        res[k + "_TBps"] = round(n * E * wrow / (res[k] * 1e-6) / 1e12, 2)
print(json.dumps(dict(config=cfg, dtype=cd, us=res)))
