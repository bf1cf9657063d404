"""GPU: fit_generator through the one-call step (Engine.fast_train_step -> ocf_train_step_rows) is
bit-identical to the general path (four library calls per step) -- weights, optimizer slots, the 16-bit
shadows and the logged history -- over two epochs with dropout, the reference's reciprocal split (NumPy's
MT19937 draws on the device) and Adagrad / Adam; and the one-call step really ran."""
import ctypes

import numpy as np
import pytest

from parity import dataset


def _run(fast, cd, opt, sparsity):
    import torch
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    data = dataset(rows=900, cols=700, nnz=40000)
    np.random.seed(21)
    rd = data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split", rng="numpy")
    om = omni_model(1, 500, data.num_cols, 128, dense_activation="sigmoid", use_causal_info=False,
                    dropout_probability=0.2, compute_dtype=cd, seed=3)
    m = om.model
    m.compile(O.Adagrad(lr=0.005, epsilon=1e-8) if opt == "adagrad" else O.Adam(lr=0.001), "mean_squared_error",
              metrics=["mae", "accurate_RMSE"])
    eng = om.engine
    eng.fast_steps = fast
    hist = []
    issued = 0
    for ep in range(2):
        gen = rd.data_gen(128, sparsity, "train", True, None, -1,
                          pass_through_input_training=sparsity == [1.0, 1.0])
        steps = gen.num_batches - 1
        n0 = eng.step_count
        h = m.fit_generator(gen, steps, epochs=1, verbose=0)
        hist.append(h.history)
        issued += eng.step_count - n0
    torch.cuda.synchronize()
    st = [t.cpu().numpy().copy() for sw, sb in eng.slots for t in sw + sb if t is not None]
    sh = [t.float().cpu().numpy() for t in eng.Wsh if t is not None]
    ready = eng._plan is not None and eng._plan.get("ready")
    return hist, m.get_weights(), st, sh, ready, issued


@pytest.mark.gpu
@pytest.mark.parametrize("cd,opt,sparsity", [("float16", "adagrad", [1.0, 1.0]), ("float32", "adagrad", [0.3, 0.7]),
                                             ("bfloat16", "adam", [0.5, 0.9])])
def test_fast_step_bit_identical(gpu, cd, opt, sparsity):
    h_f, w_f, s_f, sh_f, ready, n = _run(True, cd, opt, sparsity)
    h_g, w_g, s_g, sh_g, ready_g, n_g = _run(False, cd, opt, sparsity)
    assert ready and not ready_g and n == n_g > 0
    assert h_f == h_g and all(np.isfinite(v).all() and v[0] > 0 for h in h_f for v in h.values())
    for a, b in zip(w_f + s_f + sh_f, w_g + s_g + sh_g):
        assert np.array_equal(a, b), float(np.abs(a - b).max())


def _run_pair(pair, cd, opt, shape, jobs=False):
    import torch
    from omnidirectional_collaborative_filtering_amd import _lib
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    rows, cols, nnz, B = shape
    data = dataset(rows=rows, cols=cols, nnz=nnz)
    np.random.seed(8)
    rd = data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split", rng="numpy")
    om = omni_model(1, 500 if cd != "float32" else 200, data.num_cols, B, dense_activation="sigmoid",
                    use_causal_info=False, dropout_probability=0.2, compute_dtype=cd, seed=5)
    m = om.model
    mk = {"adagrad": lambda: O.Adagrad(lr=0.01, epsilon=1e-8), "rmsprop": lambda: O.RMSprop(lr=0.001),
          "adam": lambda: O.Adam(lr=0.001)}[opt]
    m.compile(mk(), "mean_squared_error", metrics=["mae"])
    eng = om.engine
    eng.pair_dw = pair
    if jobs:      # the row reduction as the output layer's jobs (producers), the pair form on large weights
        eng.reduce_in_decoder = False
        _lib.call("ocf_set_tuning", b"rows_dual_large", 0, None)
    gen = rd.data_gen(B, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
    _lib.call("ocf_set_tuning", b"rows_dual_count", 0, None)
    n = min(6, gen.num_batches - 1)
    try:
        h = m.fit_generator(gen, n, epochs=1, verbose=0).history
        torch.cuda.synchronize()
    finally:
        _lib.call("ocf_set_tuning", b"rows_dual_large", 1, None)
    dual = ctypes.c_int(-1)
    _lib.call("ocf_set_tuning", b"rows_dual_count", 0, ctypes.byref(dual))
    # one launch per step.  Default (the decoder did the row reduction): the dual-row form on every weight size,
    # nothing to count.  With the reduction as producer jobs: the pair form on weights of more than 170 row
    # tiles, the dual-row form with producers on smaller ones; both advance the producers' count (never cleared;
    # the host keeps its running twin; every launch on the same word)
    large = eng.Np // 128 > 170
    assert (eng.pair_state.count > 0) == (pair and jobs)
    assert dual.value == (n if pair and not (jobs and large) else 0)
    assert eng.pair_sync[0].item() == eng.pair_state.count and eng.pair_state.count % ((eng.Bp + 3) // 4) == 0
    st = [t.cpu().numpy().copy() for sw, sb in eng.slots for t in sw + sb if t is not None]
    sh = [t.float().cpu().numpy() for t in eng.Wsh if t is not None]
    return h, m.get_weights(), st, sh, eng._rtag_live


@pytest.mark.gpu
@pytest.mark.parametrize("cd,opt,shape", [
    ("float16", "adagrad", (2000, 40000, 120000, 256)),   # sparse weight rows: live-row records, 12 parts
    ("bfloat16", "adagrad", (1000, 22000, 500000, 256)),  # ~5 entries per weight row: LONG, records
    ("float32", "rmsprop", (1200, 30000, 150000, 128)),
    ("float16", "adam", (2000, 40000, 120000, 256)),
    ("bfloat16", "adagrad", (1500, 3000, 120000, 256))])  # small dense weight: two launches (no records)
@pytest.mark.parametrize("jobs", [False, True])
def test_pair_launch_bit_identical(gpu, cd, opt, shape, jobs):
    """ocf_gemm_pair in one launch (the dual-row form; with the row reduction as the output layer's jobs the
    pair form on large weights, dW_in's workgroups waiting in the kernel for it) against the two ocf_gemm
    launches: identical history, weights, slots and shadows"""
    a = _run_pair(True, cd, opt, shape, jobs)
    b = _run_pair(False, cd, opt, shape, jobs)
    assert a[0] == b[0] and a[4] == b[4]
    for x, y in zip(a[1] + a[2] + a[3], b[1] + b[2] + b[3]):
        assert np.array_equal(x, y), float(np.abs(x - y).max())
