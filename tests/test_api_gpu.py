"""GPU: the drop-in surfaces end to end -- train.py driver, Keras-style fit on dense arrays
(train_jester.py:78-79), predict, train_on_batch on user arrays vs the generator fast path,
checkpoint save/load."""
import numpy as np
import pytest

from oracle.batch_oracle import scatter_rows_numpy
from oracle.model_oracle import OmniOracle


def _data(rows=600, cols=200, nnz=9000, seed=2):
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    r, c, v = synthetic_ratings(rows, cols, nnz, half_stars=True, seed=seed)
    return split_ratings(r, c, v, rows, cols, rng=np.random.RandomState(seed))


@pytest.mark.gpu
def test_trainer_end_to_end_vs_oracle(gpu, tmp_path):
    """train.py driver on BASELINE configs[0] (ML-100K-shaped I-AutoRec, 1 x 500 sigmoid, dropout 0.2,
    Adagrad 0.005, batch 128, exact fp32): the early-stopping decisions replayed from its validation
    history (train.py:147-177), a checkpoint for exactly the improving epochs (never the first), the
    tested model = the best checkpoint (train.py:181-199), and compute_full_RMSE (train.py:225-255)
    equal to the oracle's on that checkpoint's weights over the same test batches (1e-5)"""
    import os
    from safetensors.numpy import load_file
    from omnidirectional_collaborative_filtering_amd import train
    from omnidirectional_collaborative_filtering_amd.dataset import synthetic_fixed_split
    cfg = dict(train.DEFAULTS)
    cfg.update(synthetic="ml100k", max_epochs=4, batch_size=128, num_hidden_units=500, patience=0,
               model_save_path=str(tmp_path), compute_dtype="float32", seed=4)
    out = train.run(cfg)
    st = train.EarlyStopper(0)
    saved, epochs = [], 0
    for i, v in enumerate(out["val_history"]):
        a = st.update(i, [v])
        epochs = i + 1
        if a == "save":
            saved.append(i + 1)
        if a == "stop":
            break
    assert out["epochs_run"] == epochs and out["best_epoch"] == st.best_epoch + 1
    files = sorted(f for f in os.listdir(str(tmp_path)) if f.endswith(".safetensors"))
    assert len(files) == len(saved) and all(("_epoch_%d_" % e) in f for e, f in zip(sorted(saved), files))
    assert 1 not in saved
    if not saved:
        assert out["tested_checkpoint"] is None
        return
    assert "_epoch_%d_" % out["best_epoch"] in out["tested_checkpoint"]
    t = load_file(out["tested_checkpoint"])
    w = [t["param/%d" % j] for j in range(4)]
    data = synthetic_fixed_split("ml100k", seed=0)
    N = data.num_cols
    ora = OmniOracle([N, 500, N], activation="sigmoid").set_params(w[0::2], w[1::2])
    sse, cnt = 0.0, 0
    for rows in out["manual_test_rows"]:
        _, _, x, _, _ = scatter_rows_numpy(data.test_in.row_ptr, data.test_in.col, data.test_in.val, rows, N, aux=-1.0)
        _, mo, _, tt, _ = scatter_rows_numpy(data.test_tgt.row_ptr, data.test_tgt.col, data.test_tgt.val, rows, N,
                                             aux=-1.0)
        y, _ = ora.forward(x, mo)
        sse += float(((y - tt) ** 2).sum())
        cnt += int(data.test_tgt.row_lengths()[rows].sum())
    assert abs(out["manual_test_RMSE"] - np.sqrt(sse / cnt)) <= 1e-5


@pytest.mark.gpu
def test_predict_matches_oracle(gpu):
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    rng = np.random.RandomState(0)
    B, N, H = 128, 150, 40
    om = omni_model(2, H, N, B, dense_activation="tanh", use_causal_info=True, compute_dtype="float32", seed=2)
    x = rng.rand(B, N) * (rng.rand(B, N) < 0.1)
    obs = -1.0 * (x != 0)
    mask = -1.0 * (rng.rand(B, N) < 0.2)
    y = om.model.predict([x, obs, mask]).cpu().numpy()
    w = om.model.get_weights()
    ora = OmniOracle([2 * N, H, H, N], activation="tanh").set_params(w[0::2], w[1::2])
    ref, _ = ora.forward(np.concatenate([x, obs], 1), mask)
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_dense_train_on_batch_equals_generator_path(gpu):
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    from omnidirectional_collaborative_filtering_amd.optimizers import Adagrad
    data = _data()
    N = data.num_cols
    np.random.seed(9)
    rd = data_reader(N, 600, dataset=data, eval_mode="fixed_split")
    a = omni_model(1, 32, N, 128, "sigmoid", use_causal_info=False, compute_dtype="float32", seed=5).model
    b = omni_model(1, 32, N, 128, "sigmoid", use_causal_info=False, compute_dtype="float32", seed=5).model
    a.compile(Adagrad(lr=0.01), "mean_squared_error")
    b.compile(Adagrad(lr=0.01), "mean_squared_error")
    gen = rd.data_gen(128, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
    la = a.fit_generator(gen, 2, verbose=0).history["loss"][0]
    lbs = []
    for bi in range(2):
        _, m_out, x, t, _ = scatter_rows_numpy(data.train.row_ptr, data.train.col, data.train.val, gen.rows_host[bi],
                                               N, aux=-1.0)
        lbs.append(b.train_on_batch([x, m_out], t))
    # the generator path computes the first and last layers as row gathers over the batch's rating
    # entries, the dense path as MFMA GEMMs: the same fp32 sums in another order
    assert abs(la - np.mean(lbs)) <= 1e-5 * abs(la)
    for wa, wb in zip(a.get_weights(), b.get_weights()):
        np.testing.assert_allclose(wa, wb, rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_jester_style_fit_and_checkpoint(gpu, tmp_path):
    """train_jester.py params: 2x256 hidden, causal concat, rmsprop, reciprocal 0.5 split sampled once."""
    from omnidirectional_collaborative_filtering_amd.model import EarlyStopping, omni_model
    rng = np.random.RandomState(1)
    n, N = 1280, 100
    data = np.where(rng.rand(n, N) < 0.56, rng.uniform(-10, 10, (n, N)), 99.0)
    observed = (data != 99).astype(np.float64)
    drop = rng.choice([0, 1], size=data.shape, p=[0.5, 0.5])
    in_m, out_m = drop * observed, (1 - drop) * observed
    inputs, targets = np.where(in_m > 0, data, 0.0), np.where(out_m > 0, data, 0.0)
    om = omni_model(2, 256, N, 128, dense_activation="tanh", use_causal_info=True, compute_dtype="bfloat16", seed=3,
                    rating_range=20)
    m = om.model
    m.compile("rmsprop", "mean_squared_error", metrics=["mae", "accurate_MAE", "nMAE"])
    h = m.fit([inputs, observed, out_m], targets, batch_size=128, validation_split=0.1, epochs=4, shuffle=True,
              callbacks=[EarlyStopping(monitor="val_loss", patience=3)])
    assert h.history["loss"][-1] < h.history["loss"][0]
    assert "val_loss" in h.history and "val_nMAE" in h.history
    p = str(tmp_path / "ck.safetensors")
    m.save(p)
    w = m.get_weights()
    om2 = omni_model(2, 256, N, 128, dense_activation="tanh", use_causal_info=True, compute_dtype="bfloat16", seed=99)
    om2.model.compile("rmsprop", "mean_squared_error")
    om2.model.load(p)
    for a, b in zip(w, om2.model.get_weights()):
        np.testing.assert_array_equal(a, b)
    assert om2.model.optimizer.iterations == m.optimizer.iterations


@pytest.mark.gpu
def test_denoising_transfer_freezes_outer_layers(gpu):
    """model.py:140-170 (load_and_fix_for_denoising_autoencoders) + Keras trainable=False: a 3-layer
    model takes the outer layers of a 1-hidden-layer donor and freezes them; one Adagrad step then
    equals the oracle step restricted to the trainable (middle) layers, and the frozen weights do not
    move."""
    import numpy as np
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    from omnidirectional_collaborative_filtering_amd.optimizers import Adagrad
    from oracle.model_oracle import AdagradOracle, OmniOracle
    B, N, H = 16, 40, 12
    rng = np.random.RandomState(0)
    donor = omni_model(1, H, N, B, dense_activation="sigmoid", use_causal_info=False, compute_dtype="float32", seed=3)
    om = omni_model(2, H, N, B, dense_activation="sigmoid", use_causal_info=False, compute_dtype="float32", seed=4)
    om.load_and_fix_for_denoising_autoencoders(donor)
    assert om.engine.trainable == [False, True, False]
    w0 = om.model.get_weights()
    dw = donor.model.get_weights()
    np.testing.assert_array_equal(w0[0], dw[0])
    np.testing.assert_array_equal(w0[4], dw[2])
    om.model.compile(Adagrad(lr=0.01, epsilon=1e-8), "mean_squared_error")
    x = (rng.rand(B, N) < 0.3) * rng.randint(1, 6, size=(B, N)).astype(np.float32)
    m = -1.0 * (x != 0)
    om.model.train_on_batch([x, m], x)
    w1 = om.model.get_weights()
    ora = OmniOracle([N, H, H, N], "sigmoid", None, None, np.float64).set_params(w0[0::2], w0[1::2])
    _, _, gW, gb = ora.loss_and_grads(x, m, x)
    opt = AdagradOracle(lr=0.01, epsilon=1e-8)
    new_w, new_b = opt.step([w0[2], w0[3]], [gW[1], gb[1]])
    for i in (0, 1, 4, 5):
        np.testing.assert_array_equal(w1[i], w0[i])
    np.testing.assert_allclose(w1[2], new_w, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(w1[3], new_b, rtol=1e-5, atol=1e-6)
    om.make_trainable()
    assert om.engine.trainable == [True, True, False]


@pytest.mark.gpu
def test_predict_after_generator_training(gpu):
    """predict() on dense arrays after row-gather training steps runs the dense GEMM path on the
    arrays it was given (no stale gather tables of the last generator batch): equal to the oracle
    forward with the trained weights."""
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    from omnidirectional_collaborative_filtering_amd.optimizers import Adagrad
    data = _data()
    N = data.num_cols
    np.random.seed(4)
    rd = data_reader(N, 600, dataset=data, eval_mode="fixed_split")
    om = omni_model(1, 32, N, 128, "sigmoid", use_causal_info=False, dropout_probability=0.2,
                    compute_dtype="float32", seed=6)
    m = om.model
    m.compile(Adagrad(lr=0.01), "mean_squared_error")
    gen = rd.data_gen(128, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
    m.fit_generator(gen, 2, verbose=0)
    assert om.engine.gt is not None              # the last step took the row-gather path
    rng = np.random.RandomState(1)
    x = rng.rand(128, N) * (rng.rand(128, N) < 0.1)
    mask = -1.0 * (rng.rand(128, N) < 0.2)
    y = m.predict([x, mask]).cpu().numpy()
    w = m.get_weights()
    ref, _ = OmniOracle([N, 32, N], activation="sigmoid").set_params(w[0::2], w[1::2]).forward(x, mask)
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5)
