"""GPU: ocf_gemm_pair's hand-off counter through the C ABI (ctypes), include/ocf.h OcfPairSync.

* Two pair launches on ONE counter, the word never cleared between them, give bit for bit the state of
  the same two steps as two plain ocf_gemm launches each (the counter only grows: no reset contract).
* A counter whose host count runs ahead of its word (a caller that cleared the word behind the library's
  back) makes the input layer's workgroups give up their bounded wait: they skip their update (W1 and its
  slots untouched) and the next library call fails with the asynchronous error, once.
The argument blocks are the engine's own one-call template (Engine._plan, ocf.h OcfRowStepArgs) for the
last step of a short fit on an ML-20M-like sparse shape (more than 170 row tiles: the pair launch)."""
import ctypes

import numpy as np
import pytest

from parity import dataset


def _engine():
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    data = dataset(rows=2000, cols=40000, nnz=120000)
    np.random.seed(4)
    rd = data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split", rng="numpy")
    om = omni_model(1, 500, data.num_cols, 256, dense_activation="sigmoid", use_causal_info=False,
                    dropout_probability=0.2, compute_dtype="float16", seed=9)
    om.model.compile(O.Adagrad(lr=0.01, epsilon=1e-8), "mean_squared_error", metrics=["mae"])
    gen = rd.data_gen(256, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
    om.model.fit_generator(gen, 5, epochs=1, verbose=0)
    eng = om.engine
    assert eng._plan is not None and eng._plan.get("ready") and eng._plan["st"].pair_sync
    return eng


def _state(eng):
    ts = list(eng.W) + list(eng.b) + [t for sw, sb in eng.slots for t in sw + sb if t is not None]
    return ts + [t for t in eng.Wsh if t is not None] + list(eng.dh)


def _blocks(eng):
    from omnidirectional_collaborative_filtering_amd import _lib
    st = eng._plan["st"]
    g_out = _lib.OcfGemmArgs.from_buffer_copy(st.dw_out)
    g_out.jr = ctypes.addressof(st.jr)            # what ocf_train_step_rows passes (jr_on)
    return g_out, st.dw_in


@pytest.mark.gpu
def test_pair_twice_without_clearing_matches_two_launches(gpu):
    import torch
    from omnidirectional_collaborative_filtering_amd import _lib
    from omnidirectional_collaborative_filtering_amd.engine import cur_stream
    eng = _engine()
    g_out, g_in = _blocks(eng)
    torch.cuda.synchronize()
    s0 = [t.clone() for t in _state(eng)]
    word = torch.zeros(1, dtype=torch.int64, device="cuda")
    sync = _lib.OcfPairSync(word.data_ptr(), 0)
    for _ in range(2):
        _lib.call("ocf_gemm_pair", g_out, g_in, ctypes.addressof(sync), cur_stream())
    torch.cuda.synchronize()
    n_prod = (eng.Bp + 3) // 4
    assert sync.count == 2 * n_prod and word.item() == 2 * n_prod     # counted up, never cleared
    a = [t.clone() for t in _state(eng)]
    for t, v in zip(_state(eng), s0):
        t.copy_(v)
    for _ in range(2):
        _lib.call("ocf_gemm", g_out, cur_stream())
        _lib.call("ocf_gemm", g_in, cur_stream())
    torch.cuda.synchronize()
    b = _state(eng)
    changed = False
    for x, y, z in zip(a, b, s0):
        assert torch.equal(x, y), float((x.float() - y.float()).abs().max())
        changed |= not torch.equal(x, z)
    assert changed


@pytest.mark.gpu
def test_pair_wait_gives_up_loudly(gpu):
    import torch
    from omnidirectional_collaborative_filtering_amd import _lib
    from omnidirectional_collaborative_filtering_amd.engine import cur_stream
    eng = _engine()
    g_out, g_in = _blocks(eng)
    torch.cuda.synchronize()
    w_in = eng.W[0].clone()
    a_in = eng.slots[0][0][0].clone()
    lib = _lib.load()
    prev = ctypes.c_int32()
    _lib.call("ocf_set_tuning", b"pair_wait_polls", 2000, ctypes.byref(prev))
    try:
        word = torch.zeros(1, dtype=torch.int64, device="cuda")
        sync = _lib.OcfPairSync(word.data_ptr(), 10 ** 6)   # the host count far ahead of its word
        _lib.call("ocf_gemm_pair", g_out, g_in, ctypes.addressof(sync), cur_stream())
        torch.cuda.synchronize()
        # the input layer's rows were skipped, not updated from a stale delta
        assert torch.equal(eng.W[0], w_in) and torch.equal(eng.slots[0][0][0], a_in)
        # the next call reports it (any entry point), then the word is clear again
        rc = lib.ocf_set_tuning(b"pair_wait_polls", 2000, None)
        assert rc != 0 and b"ocf_gemm_pair" in lib.ocf_last_error()
        assert lib.ocf_set_tuning(b"pair_wait_polls", 2000, None) == 0
    finally:
        lib.ocf_set_tuning(b"pair_wait_polls", prev.value, None)
