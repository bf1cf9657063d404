"""GPU: a feature-parallel rank's gathers in the row-resident form (ocf_rank_step phases 0 / 1 as one launch each,
ocf_set_tuning "encdec_rowres") against the separate launches (encoder + RAW reduction; ocf_splitk_bias_act +
decoder + RAW reduction + stats), on one rank of a 4-way column shard with its collectives as no-ops (bench.py
--emulate-shards), skewed rows (some of them empty in the shard) and padding rows (B = 500 of 512).  Only the order
of fp32 sums differs: fp32 weights within 1e-5, 16-bit ones inside tests/parity.py's per-element envelope (units of
lr x steps: max 2, p99 0.02, p99.9 0.15), losses 1e-5 / 2e-3 relative."""
import ctypes

import numpy as np
import pytest
import torch


class _NoComm:
    class _Work:
        def wait(self):
            pass

    def __call__(self, t):
        pass

    def start(self, t):
        return self._Work()


def _run(cd, rowres, steps=5):
    from omnidirectional_collaborative_filtering_amd import _lib, optimizers as O
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    from omnidirectional_collaborative_filtering_amd.parallel import feature_shard_range
    prev = ctypes.c_int32()
    _lib.call("ocf_set_tuning", b"encdec_rowres", int(rowres), ctypes.byref(prev))
    try:
        rows, cols, nnz = 3000, 20000, 400000
        r, c, v = synthetic_ratings(rows, cols, nnz, half_stars=True, seed=12, skew=0.8)
        full = split_ratings(r, c, v, rows, cols, rng=np.random.RandomState(12))
        c0, c1 = feature_shard_range(cols, 1, 4)
        data = full.column_shard(c0, c1)
        np.random.seed(5)
        rd = data_reader(data.num_cols, full.train.n_rows, dataset=data, eval_mode="fixed_split", rng="numpy")
        om = omni_model(1, 500, data.num_cols, 500, dense_activation="sigmoid", use_causal_info=False,
                        dropout_probability=0.2, compute_dtype=cd, seed=7, shard=(c0, c1, cols), comm=_NoComm())
        m = om.model
        m.compile(O.Adagrad(lr=0.005, epsilon=1e-8), "mean_squared_error")
        gen = rd.data_gen(500, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
        losses = [m.fit_generator(gen, 1, epochs=1, verbose=0).history["loss"][0] for _ in range(steps)]
        torch.cuda.synchronize()
        eng = om.engine
        assert eng.step_paths["one_call"] >= steps - 2       # the rank template (ocf_rank_step) took the late steps
        return losses, [t.detach().float().cpu().numpy().copy() for t in eng.W + eng.b]
    finally:
        _lib.call("ocf_set_tuning", b"encdec_rowres", prev.value, None)


@pytest.mark.gpu
@pytest.mark.parametrize("cd", ["float32", "float16", "bfloat16"])
def test_rank_rowres_matches_separate_launches(gpu, cd):
    l0, w0 = _run(cd, 0)
    l1, w1 = _run(cd, 1)
    tol = 1e-5 if cd == "float32" else 2e-3
    for a, b in zip(l0, l1):
        assert abs(a - b) <= tol * abs(a), (l0, l1)
    # (the two forms sum in different orders: a bit-identical result would mean one of them did not run)
    assert any(not np.array_equal(a, b) for a, b in zip(w0, w1))
    unit = 1.0 if cd == "float32" else 0.005 * 5
    for a, b in zip(w0, w1):
        d = np.abs(a - b).ravel() / unit
        if cd == "float32":
            assert d.max() <= 1e-5, float(d.max())
        else:
            assert d.max() <= 2.0 and np.quantile(d, 0.99) <= 0.02 and np.quantile(d, 0.999) <= 0.15, \
                (float(d.max()), float(np.quantile(d, 0.99)), float(np.quantile(d, 0.999)))
