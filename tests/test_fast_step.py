"""CPU: the one-call training step (Engine.fast_train_step -> ocf_train_step_rows) issues exactly the
argument blocks the general path builds.  The library is stubbed (no GPU here: every call records and
returns 0) and the engine lives on host tensors, so the test sees the pointers and scalars of every call.
For each step after the template is verified, the template rewritten for the step (the batch's table
pointers from BatchGenerator.step_fields, the Philox stream, the stats slot, the optimizer constants) is
compared byte for byte with the four argument blocks the general path records for the same step --
across epochs (new generators), row-list windows, the reference's reciprocal split with its NumPy draws,
dropout, and optimizers whose constants change per step (Adam's bias correction, Keras decay)."""
import contextlib
import ctypes

import numpy as np
import pytest
import torch

from omnidirectional_collaborative_filtering_amd import _lib


@pytest.fixture
def stubbed(monkeypatch):
    _lib.load()
    seen = []

    def fake_call(name, *args):
        if name == "ocf_train_step_rows":
            st = args[0]
            seen.append(ctypes.string_at(ctypes.addressof(st), ctypes.sizeof(st)))
        if name == "ocf_rank_step" and args[1] == 0:
            seen.append(ctypes.string_at(ctypes.addressof(args[0]), ctypes.sizeof(args[0])))
        return 0
    monkeypatch.setattr(_lib, "call", fake_call)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    from omnidirectional_collaborative_filtering_amd import data_reader as DR
    from omnidirectional_collaborative_filtering_amd import engine as E
    monkeypatch.setattr(E, "cur_stream", lambda: None)
    monkeypatch.setattr(DR, "cur_stream", lambda: None)
    monkeypatch.setattr(DR, "_rng_stream", lambda dev: None)
    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())
    monkeypatch.setattr(DR, "ROWLIST_MAX_BATCHES", 3)     # several row-list windows per epoch
    return seen


def _model(opt, dropout, data):
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    om = omni_model(1, 100, data.num_cols, 32, dense_activation="sigmoid", use_causal_info=False,
                    dropout_probability=dropout, compute_dtype="float16", seed=7, device=torch.device("cpu"))
    o = {"adagrad": lambda: O.Adagrad(lr=0.005, epsilon=1e-8), "adagrad_decay": lambda: O.Adagrad(lr=0.005, decay=0.01),
         "adam": lambda: O.Adam(lr=0.001), "rmsprop": lambda: O.RMSprop(lr=0.001)}[opt]()
    om.model.compile(o, "mean_squared_error")
    return om


@pytest.mark.parametrize("opt,dropout,sparsity,pair,encdec", [("adagrad", 0.2, [1.0, 1.0], True, True),
                                                              ("adagrad", None, [0.3, 0.7], True, False),
                                                              ("adam", 0.2, [0.5, 0.9], True, True),
                                                              ("adagrad_decay", 0.2, [1.0, 1.0], False, True),
                                                              ("rmsprop", None, [1.0, 1.0], False, False)])
def test_fast_step_blocks_equal_general_path(stubbed, opt, dropout, sparsity, pair, encdec):
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    r, c, v = synthetic_ratings(400, 300, 9000, half_stars=True, seed=3)
    data = split_ratings(r, c, v, 400, 300, rng=np.random.RandomState(3), dup_free=True)
    np.random.seed(5)
    rd = data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split", rng="numpy",
                     device=torch.device("cpu"))
    om = _model(opt, dropout, data)
    eng = om.engine
    eng.pair_dw = pair
    eng.fuse_enc_dec = encdec           # the encoder and the decoder as one launch (ocf_gather_encdec) or two
    checked = fast = 0
    for epoch in range(5):
        gen = rd.data_gen(32, sparsity, "train", True, None, -1, pass_through_input_training=False)
        while True:
            bi = gen.next_batch_index()
            if bi is None:
                break
            pl = eng._plan
            f = gen.step_fields(bi, eng.Np)
            if pl is not None and pl.get("ready") and eng._fast_key(gen) == pl["key"] and f is not None \
                    and eng._fits(pl, f):
                if (bi + epoch) % 3 == 0:      # the real one-call step (keeps the engine's counters moving)
                    assert eng.fast_train_step(gen, bi)
                    fast += 1
                    continue
                cand = dict(pl, st=_lib.OcfRowStepArgs.from_buffer_copy(pl["st"]))
                eng._bind(cand)
                eng._grow_stats(eng.n_stats + 1)
                eng._rewrite(cand, f, eng._per_step())
                calls = eng._recorded_step(gen, bi)
                assert tuple(n for n, _ in calls) == eng._STEP_CALLS[(0 if pair else 1) + (2 if encdec else 0)]
                assert eng._same(cand, calls), (epoch, bi)
                checked += 1
            else:
                assert eng.fast_train_step(gen, bi)
    assert checked >= 12 and fast >= 5, (checked, fast)
    assert len(stubbed) == fast


def test_fast_step_declines_other_layouts(stubbed):
    """a step the template does not cover stays on the general path: two hidden layers, l2, frozen layers,
    the valid split"""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    r, c, v = synthetic_ratings(400, 300, 9000, half_stars=True, seed=3)
    data = split_ratings(r, c, v, 400, 300, rng=np.random.RandomState(3), dup_free=True)
    np.random.seed(5)
    rd = data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split", rng="numpy",
                     device=torch.device("cpu"))
    cpu = torch.device("cpu")
    two = omni_model(2, 64, data.num_cols, 32, dense_activation="sigmoid", use_causal_info=False, device=cpu)
    l2 = omni_model(1, 64, data.num_cols, 32, dense_activation="sigmoid", use_causal_info=False, device=cpu,
                    l2_weight_regulatization=1e-4)
    frozen = omni_model(1, 64, data.num_cols, 32, dense_activation="sigmoid", use_causal_info=False, device=cpu)
    for om in (two, l2, frozen):
        om.model.compile(O.Adagrad(lr=0.005), "mean_squared_error")
    frozen.engine.trainable[0] = False
    for om in (two, l2, frozen):
        gen = rd.data_gen(32, [1.0, 1.0], "train", True, None, -1)
        for _ in range(4):
            assert not om.engine.fast_train_step(gen, gen.next_batch_index())
    vg = rd.data_gen(32, None, "valid", True, None, -1)
    ok = _model("adagrad", None, data).engine
    assert not ok.fast_train_step(vg, vg.next_batch_index())
    assert not stubbed


class _Comm:
    """feature-parallel collectives of one rank alone (no-ops with the real call shape: comm(t) and the
    asynchronous start(t).wait())"""

    class _W:
        def wait(self):
            pass

    def __call__(self, t):
        pass

    def start(self, t):
        return self._W()


@pytest.mark.parametrize("opt,dropout,sparsity", [("adagrad", 0.2, [1.0, 1.0]), ("rmsprop", None, [0.3, 0.7])])
def test_rank_step_blocks_equal_general_path(stubbed, opt, dropout, sparsity):
    """the feature-parallel rank step's template (ocf.h OcfRankStepArgs, Engine._fast_rank_step) rewritten for
    each step equals the ten argument blocks the general path builds for it, byte for byte, across epochs,
    row-list windows and the reciprocal split; the real one-call steps issue four ocf_rank_step phases"""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    from omnidirectional_collaborative_filtering_amd.parallel import feature_shard_range
    r, c, v = synthetic_ratings(400, 600, 12000, half_stars=True, seed=3)
    data = split_ratings(r, c, v, 400, 600, rng=np.random.RandomState(3), dup_free=True)
    c0, c1 = feature_shard_range(data.num_cols, 1, 4)
    ds = data.column_shard(c0, c1)
    np.random.seed(5)
    rd = data_reader(ds.num_cols, data.train.n_rows, dataset=ds, eval_mode="fixed_split", rng="numpy",
                     device=torch.device("cpu"))
    om = omni_model(1, 100, ds.num_cols, 32, dense_activation="sigmoid", use_causal_info=False,
                    dropout_probability=dropout, compute_dtype="float16", seed=7, device=torch.device("cpu"),
                    shard=(c0, c1, data.num_cols), comm=_Comm())
    om.model.compile({"adagrad": lambda: O.Adagrad(lr=0.005), "rmsprop": lambda: O.RMSprop(lr=0.001)}[opt](),
                     "mean_squared_error")
    eng = om.engine
    b = lambda x: ctypes.string_at(ctypes.addressof(x), ctypes.sizeof(x))
    checked = fast = 0
    for epoch in range(5):
        gen = rd.data_gen(32, sparsity, "train", True, None, -1, pass_through_input_training=sparsity[0] >= 1.0)
        while True:
            bi = gen.next_batch_index()
            if bi is None:
                break
            pl = eng._rplan
            f = gen.step_fields(bi, eng.Np)
            if pl is not None and pl.get("ready") and eng._rank_key(gen) == pl["key"] and f is not None \
                    and eng._rank_fits(pl, f):
                if (bi + epoch) % 3 == 0:
                    assert eng.fast_train_step(gen, bi)
                    fast += 1
                    continue
                st = _lib.OcfRankStepArgs.from_buffer_copy(pl["st"])
                eng._grow_stats(eng.n_stats + 1)
                eng._rank_rewrite(st, f, eng._rank_stream(eng.step_count), eng._stats_row(eng.n_stats), pl["live"])
                calls = eng._recorded_step(gen, bi)
                assert tuple(n for n, _ in calls) == eng._RANK_CALLS
                assert b(st) == b(eng._rank_template(pl["key"], calls)["st"]), (epoch, bi)
                checked += 1
            else:
                assert eng.fast_train_step(gen, bi)
    assert checked >= 12 and fast >= 5, (checked, fast)



def test_row_list_window_args(stubbed, monkeypatch):
    """BatchGenerator.prepare_row_lists: a window of consecutive batches points sel / ebase into the epoch's device
    tables and rebases the entry offsets with ebase0 (nothing staged); any other selection is staged and starts at
    entry 0; both pass the list-length bound and the entry count the library picks its passes by"""
    from omnidirectional_collaborative_filtering_amd import data_reader as DR
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    r, c, v = synthetic_ratings(400, 300, 9000, half_stars=True, seed=3)
    data = split_ratings(r, c, v, 400, 300, rng=np.random.RandomState(3), dup_free=True)
    np.random.seed(5)
    rd = DR.data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split", rng="numpy",
                        device=torch.device("cpu"))
    got = {}

    def fake_call(name, *args):
        if name in ("ocf_epoch_row_lists", "ocf_epoch_scatter"):
            a = args[0] if name == "ocf_epoch_row_lists" else args[1]
            got[name] = type(a).from_buffer_copy(a)
        return 0
    monkeypatch.setattr(_lib, "call", fake_call)
    gen = rd.data_gen(32, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
    gen._start()
    assert gen.num_batches >= 6
    n_cols = 384
    eb = np.concatenate([[0], np.cumsum(gen.nnz1)])
    for sel, window in (([2, 3, 4], True), ([4, 1], False), ([5, 3, 4, 3], True)):
        gen.prepare_row_lists(n_cols, sel)
        s = sorted(set(sel))
        el, es = got["ocf_epoch_row_lists"], got["ocf_epoch_scatter"]
        ep = gen._ep_tabs
        E = int(gen.nnz1[s].sum())
        assert el.n_sel == es.n_sel == len(s) and el.entries == E and el.max_list == gen.B
        assert el.sel == es.sel and el.ebase == es.ebase and el.ebase0 == es.ebase0
        if window:
            assert el.sel == ep["sel_dev"].data_ptr() + 4 * s[0]
            assert el.ebase == ep["ebase_dev"].data_ptr() + 8 * s[0]
            assert el.ebase0 == eb[s[0]]
        else:
            assert el.ebase0 == 0
            staged = ctypes.cast(el.ebase, ctypes.POINTER(ctypes.c_int64))
            assert [staged[i] for i in range(len(s) + 1)] == [0] + list(np.cumsum(gen.nnz1[s]))
        rl = gen._rl
        assert rl["slot"] == {b: i for i, b in enumerate(s)}
        np.testing.assert_array_equal(rl["ebase_host"], np.concatenate([[0], np.cumsum(gen.nnz1[s])]))
