# Which host calls issue PyTorch fill kernels inside generator training steps (torch.profiler with
# Python stacks over two steady-state steps of the ML-20M bench workload): python tools/find_fills.py
import sys
import numpy as np
import torch
from torch.profiler import ProfilerActivity, profile
sys.path.insert(0, '.')
from omnidirectional_collaborative_filtering_amd import optimizers as O
from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
from omnidirectional_collaborative_filtering_amd.dataset import synthetic_fixed_split
from omnidirectional_collaborative_filtering_amd.model import omni_model
cfg = sys.argv[1] if len(sys.argv) > 1 else "ml20m"
data = synthetic_fixed_split(cfg, seed=0)
np.random.seed(1234)
dev = torch.device("cuda", 0)
rd = data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split", rng="device", device=dev)
om = omni_model(1, 500, data.num_cols, 256, dense_activation="sigmoid", use_causal_info=False, dropout_probability=0.2,
                compute_dtype="float16", seed=7, device=dev)
m = om.model
m.compile(O.Adagrad(lr=0.005, epsilon=1e-8), "mean_squared_error", metrics=["mae"])
eng = om.engine
gen = rd.data_gen(256, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
gen._start()
eng.enable_timers(True, only=["dW_out"])
for i in range(6):
    m._load(None, gen, i)
    eng.train_step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    for i in range(6, 8):
        m._load(None, gen, i)
        eng.train_step()
    torch.cuda.synchronize()
for ev in prof.events():
    if ev.name in ("aten::fill_", "aten::zero_", "aten::zeros", "aten::copy_", "aten::empty", "aten::index", "aten::select"):
        print("===", ev.name, [str(s) for s in ev.stack[:8]])
print("done")
