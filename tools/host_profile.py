# Host-side cost of the generator training step (cProfile over 200 steps of a small config, where the step
# is host-bound): python tools/host_profile.py [config]
import cProfile
import pstats
import sys

import numpy as np
import torch
sys.path.insert(0, '.')
from omnidirectional_collaborative_filtering_amd import optimizers as O
from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
from omnidirectional_collaborative_filtering_amd.dataset import synthetic_fixed_split
from omnidirectional_collaborative_filtering_amd.model import omni_model
cfg = sys.argv[1] if len(sys.argv) > 1 else "ml100k"
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
nb = gen.num_batches
for i in range(5):
    m._load(None, gen, i % nb)
    eng.train_step()
torch.cuda.synchronize()

def run():
    for i in range(200):
        m._load(None, gen, i % nb)
        eng.train_step()
    torch.cuda.synchronize()

pr = cProfile.Profile()
pr.enable()
run()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
