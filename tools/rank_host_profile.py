"""Host cost of the feature-parallel rank step's one-call path (Engine._fast_rank_step) on the CPU, with the
library stubbed (every call returns at once) and the collectives no-ops: the Python part of
host_issue_ms_per_step, without the HIP launch API.  Diagnostic tool.
    python tools/rank_host_profile.py [--steps 400] [--profile 1]"""
import argparse
import contextlib
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnidirectional_collaborative_filtering_amd import _lib  # noqa: E402


class _Comm:
    class _W:
        def wait(self):
            pass

    def __call__(self, t):
        pass

    def start(self, t):
        return self._W()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--profile", type=int, default=1)
    a = ap.parse_args()
    _lib.load()
    _lib.call = lambda name, *args: 0
    torch.cuda.is_available = lambda: True
    from omnidirectional_collaborative_filtering_amd import data_reader as DR
    from omnidirectional_collaborative_filtering_amd import engine as E
    E.cur_stream = lambda: None
    DR.cur_stream = lambda: None
    DR._rng_stream = lambda dev: None
    torch.cuda.stream = lambda s: contextlib.nullcontext()
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    from omnidirectional_collaborative_filtering_amd.parallel import feature_shard_range
    r, c, v = synthetic_ratings(4000, 2400, 120000, half_stars=True, seed=3)
    data = split_ratings(r, c, v, 4000, 2400, rng=np.random.RandomState(3), dup_free=True)
    c0, c1 = feature_shard_range(data.num_cols, 1, 8)
    ds = data.column_shard(c0, c1)
    np.random.seed(5)
    rd = data_reader(ds.num_cols, data.train.n_rows, dataset=ds, eval_mode="fixed_split", rng="numpy",
                     device=torch.device("cpu"))
    om = omni_model(1, 500, ds.num_cols, 256, dense_activation="sigmoid", use_causal_info=False,
                    dropout_probability=0.2, compute_dtype="float16", seed=7, device=torch.device("cpu"),
                    shard=(c0, c1, data.num_cols), comm=_Comm())
    om.model.compile(O.Adagrad(lr=0.005), "mean_squared_error")
    eng = om.engine
    done, t_fast, n_fast = 0, 0.0, 0
    prof = cProfile.Profile() if a.profile else None
    rec = [0]
    orig = eng._recorded_step

    def counted(*x, **k):
        rec[0] += 1
        return orig(*x, **k)
    eng._recorded_step = counted
    while done < a.steps:
        gen = rd.data_gen(256, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
        while done < a.steps:
            bi = gen.next_batch_index()
            if bi is None:
                break
            ready = eng._rplan is not None and eng._rplan.get("ready")
            r0 = rec[0]
            t0 = time.perf_counter()
            if ready and prof:
                prof.enable()
            eng.fast_train_step(gen, bi)
            if ready and prof:
                prof.disable()
            if ready and rec[0] == r0:          # the one-call path (no recorded general step)
                t_fast += time.perf_counter() - t0
                n_fast += 1
            done += 1
    print({"one_call_steps": n_fast, "us_per_step": round(t_fast / max(n_fast, 1) * 1e6, 1)})
    if prof:
        pstats.Stats(prof).sort_stats("cumulative").print_stats(18)


if __name__ == "__main__":
    main()
