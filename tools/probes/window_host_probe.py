"""Host time of a row-list window's prelude (BatchGenerator.prepare_row_lists) by part, the library calls stubbed
after a first real build (diagnostic: what the timed region's first launch waits for).
    python tools/probes/window_host_probe.py ml20m|ml100k|ml1m"""
import cProfile
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from omnidirectional_collaborative_filtering_amd import _lib                      # noqa: E402
from omnidirectional_collaborative_filtering_amd import data_reader as drm        # noqa: E402
from omnidirectional_collaborative_filtering_amd.dataset import synthetic_fixed_split  # noqa: E402


def main():
    cfg = sys.argv[1]
    data = synthetic_fixed_split(cfg, seed=0)
    np.random.seed(1234)
    rd = drm.data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split", rng="numpy",
                         device="cuda")
    gen = rd.data_gen(256, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
    gen._start()
    Np = -(-data.num_cols // 128) * 128
    nb = gen.num_batches
    sel = [(5 + i) % nb for i in range(20)]
    gen.prepare_row_lists(Np, sel)
    torch.cuda.synchronize()
    real = _lib.call
    _lib.call = lambda name, *a: 0                 # the launches themselves: stubbed from here on
    ts = []
    for _ in range(300):
        t0 = time.perf_counter()
        gen.prepare_row_lists(Np, sel)
        ts.append((time.perf_counter() - t0) * 1e6)
    print(cfg, "python part of prepare_row_lists: median %.1f us" % np.median(ts), gen.rl_host_us)
    cProfile.runctx("for _ in range(3000): gen.prepare_row_lists(Np, sel)", globals(), locals(), "/tmp/wh.out")
    pstats.Stats("/tmp/wh.out").sort_stats("tottime").print_stats(14)
    _lib.call = real
    # the real calls' host time (launches included), GPU drained between builds
    ts = []
    for _ in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gen.prepare_row_lists(Np, sel)
        ts.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    print(cfg, "with the library calls: median %.1f us" % np.median(ts), gen.rl_host_us)


if __name__ == "__main__":
    main()
