"""Time the model ABI (ocf_forward / ocf_masked_mse / ocf_backward / ocf_opt_step via model_abi.ModelABI) on dense
data_gen batches (the reference's batch format, data_reader.py:354-361), beside the engine's dense path
(Model.train_on_batch on the same device arrays): one JSON line.

    python tools/model_abi_bench.py [ml1m|ml100k|ml1m_u] [dtype]
"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from omnidirectional_collaborative_filtering_amd import optimizers as O  # noqa: E402
from omnidirectional_collaborative_filtering_amd.data_reader import data_reader  # noqa: E402
from omnidirectional_collaborative_filtering_amd.dataset import synthetic_fixed_split  # noqa: E402
from omnidirectional_collaborative_filtering_amd.model import omni_model  # noqa: E402
from omnidirectional_collaborative_filtering_amd.model_abi import ModelABI  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "ml1m"
dtype = sys.argv[2] if len(sys.argv) > 2 else "bfloat16"
B, H, STEPS, WARM = 256, 500, 40, 5
data = synthetic_fixed_split(cfg, seed=0)
N = data.num_cols
dev = torch.device("cuda", 0)
np.random.seed(1234)
rd = data_reader(N, data.train.n_rows, dataset=data, eval_mode="fixed_split", rng="device", device=dev)
gen = rd.data_gen(B, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
batches = []
for _ in range(min(20, gen.num_batches)):
    (x, mo), t = gen.next()
    batches.append((x.contiguous(), mo.contiguous(), t.contiguous()))
nnz = [int((b[0] != 0).sum()) for b in batches]


def timed(fn):
    for i in range(WARM):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(STEPS):
        fn(WARM + i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / STEPS * 1e3


abi = ModelABI(N, [H], B, activation="sigmoid", dropout=0.2, compute_dtype=dtype, seed=7,
               optimizer=O.Adagrad(lr=0.005, epsilon=1e-8))


def abi_step(i):
    x, mo, t = batches[i % len(batches)]
    abi.train_on_batch([x], mo, t)


om = omni_model(1, H, N, B, dense_activation="sigmoid", use_causal_info=False, dropout_probability=0.2,
                compute_dtype=dtype, seed=7, device=dev)
om.model.compile(O.Adagrad(lr=0.005, epsilon=1e-8), "mean_squared_error", metrics=["mae"])


def eng_step(i):
    x, mo, t = batches[i % len(batches)]
    om.model.train_on_batch([x, mo], t)


ms_abi = timed(abi_step)
ms_eng = timed(eng_step)
per = float(np.mean(nnz))
print(json.dumps({"config": cfg, "dtype": dtype, "batch": B, "hidden": H, "N": N, "steps": STEPS,
                  "model_abi_ms_per_step": round(ms_abi, 4), "model_abi_ratings_per_s": round(per / ms_abi * 1e3, 1),
                  "engine_dense_ms_per_step": round(ms_eng, 4),
                  "engine_dense_ratings_per_s": round(per / ms_eng * 1e3, 1),
                  "note": "dense [B][N] batches resident in HBM (data_gen arrays); model ABI = five library calls "
                          "per step (raw fp32 gradients + elementwise Adagrad), engine = fused-optimizer dense path"}))
