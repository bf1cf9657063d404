"""Training-step parity: GPU engine (fit_generator fast path) vs the NumPy restatement of the
Keras 2.0.4 arithmetic (oracle/model_oracle.py), identical inputs and initial weights.

Bar (north_star): masked-RMSE within 1e-5 in the exact-fp32 mode; per-step loss within 1e-5
relative.  f16 / bf16 MFMA modes get looser, stated tolerances."""
import numpy as np
import pytest

from oracle.batch_oracle import scatter_rows_numpy
from oracle.model_oracle import AdagradOracle, AdamOracle, OmniOracle, RMSpropOracle


def _dataset(rows=700, cols=333, nnz=14000, seed=5):
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    r, c, v = synthetic_ratings(rows, cols, nnz, half_stars=True, seed=seed)
    return split_ratings(r, c, v, rows, cols, rng=np.random.RandomState(seed))


def _dense(csr, rows, N, aux):
    return scatter_rows_numpy(csr.row_ptr, csr.col, csr.val, rows, N, aux=aux)


def _oracle_opt(name):
    return {"adagrad": lambda: AdagradOracle(lr=0.005, epsilon=1e-8),
            "rmsprop": lambda: RMSpropOracle(lr=0.001),
            "adam": lambda: AdamOracle(lr=0.001)}[name]()


def _our_opt(name):
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    return {"adagrad": lambda: O.Adagrad(lr=0.005, epsilon=1e-8), "rmsprop": lambda: O.RMSprop(lr=0.001),
            "adam": lambda: O.Adam(lr=0.001)}[name]()


def run_parity(compute_dtype, opt_name, layers, act, steps=4, B=128, H=100, aux_type=None, causal=False,
               gather=True, sparse_dw=None):
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    data = _dataset()
    N = data.num_cols
    np.random.seed(77)
    rd = data_reader(N, 700, dataset=data, eval_mode="fixed_split")
    om = omni_model(layers, H, N, B, dense_activation=act, use_causal_info=causal, compute_dtype=compute_dtype,
                    seed=11)
    m = om.model
    om.engine.use_sparse = gather
    if sparse_dw is not None:
        om.engine.sparse_dw = sparse_dw
    m.compile(_our_opt(opt_name), "mean_squared_error", metrics=["mae", "accurate_MSE", "accurate_RMSE"])
    w0 = m.get_weights()
    gen = rd.data_gen(B, [1.0, 1.0], "train", True, aux_type, -1, pass_through_input_training=True)
    hist = m.fit_generator(gen, steps, epochs=1, verbose=0)
    w_gpu = m.get_weights()
    # oracle on the same rows (the generator exposes its epoch plan)
    k = 1 + int(causal)
    ora = OmniOracle([k * N] + [H] * layers + [N], activation=act, dtype=np.float64).set_params(w0[0::2], w0[1::2])
    opt = _oracle_opt(opt_name)
    losses = []
    for bi in range(steps):
        m_in, m_out, x, t, m_miss = _dense(data.train, gen.rows_host[bi], N, -1.0)
        xin = np.concatenate([x, m_miss if aux_type == "causal" else m_in], 1) if causal else x
        loss, _, gW, gb = ora.loss_and_grads(xin, m_out, t)
        losses.append(loss)
        flat = opt.step(ora.params(), [g for pair in zip(gW, gb) for g in pair])
        ora.set_flat(flat)
    # masked test RMSE of both models (train.py:225-255) on identical test batches
    np.random.seed(99)
    tgen = rd.data_gen(B, None, "test", True, aux_type, -1, return_target_count=True)
    nb = rd.test_set_size // B
    sse, cnt = m.evaluate_sse(tgen, nb)
    rmse_gpu = np.sqrt(sse / cnt)
    sse_o, cnt_o = 0.0, 0
    for bi in range(nb):
        rows = tgen.rows_host[bi]
        mi, _, x, _, mm = _dense(data.test_in, rows, N, -1.0)
        _, mo, _, t, mm2 = _dense(data.test_tgt, rows, N, -1.0)
        miss = np.maximum(np.abs(mm), np.abs(mm2)) * -1.0
        xin = np.concatenate([x, miss if aux_type == "causal" else mi], 1) if causal else x
        y, _ = ora.forward(xin, mo)
        sse_o += float(((y - t) ** 2).sum())
        cnt_o += int(data.test_tgt.row_lengths()[rows].sum())
    rmse_o = np.sqrt(sse_o / cnt_o)
    assert cnt == cnt_o
    return hist.history["loss"][0], float(np.mean(losses)), rmse_gpu, rmse_o, w_gpu, ora


@pytest.mark.gpu
@pytest.mark.parametrize("opt_name", ["adagrad", "rmsprop", "adam"])
def test_fp32_parity_one_hidden(gpu, opt_name):
    loss_g, loss_o, r_g, r_o, w, ora = run_parity("float32", opt_name, 1, "sigmoid")
    assert abs(loss_g - loss_o) <= 1e-5 * abs(loss_o), (loss_g, loss_o)
    assert abs(r_g - r_o) <= 1e-5, (r_g, r_o)
    for wg, wo in zip(w[0::2], ora.W):
        d = np.abs(wg - wo)
        assert np.quantile(d, 0.999) < 1e-5, np.quantile(d, 0.999)


@pytest.mark.gpu
def test_fp32_parity_two_hidden_tanh_causal(gpu):
    loss_g, loss_o, r_g, r_o, w, ora = run_parity("float32", "rmsprop", 2, "tanh", aux_type="causal", causal=True,
                                                 H=96)
    assert abs(loss_g - loss_o) <= 1e-5 * abs(loss_o), (loss_g, loss_o)
    assert abs(r_g - r_o) <= 1e-5, (r_g, r_o)


@pytest.mark.gpu
@pytest.mark.parametrize("cd,tol", [("float16", 2e-3), ("bfloat16", 1e-2)])
def test_low_precision_close(gpu, cd, tol):
    loss_g, loss_o, r_g, r_o, w, ora = run_parity(cd, "adagrad", 1, "sigmoid")
    assert abs(loss_g - loss_o) <= tol * abs(loss_o), (loss_g, loss_o)
    assert abs(r_g - r_o) <= tol * r_o, (r_g, r_o)


@pytest.mark.gpu
@pytest.mark.parametrize("gather,sparse_dw", [(False, None), (True, False), (True, True)])
def test_fp32_parity_operand_paths(gpu, gather, sparse_dw):
    """The three first/last-layer operand paths of the generator step -- dense MFMA GEMMs
    (gather off), row gathers with dense weight-gradient operands (the feature-parallel global
    batch), row gathers with sparse-A weight gradients (short K) -- each meet the fp32 bar."""
    loss_g, loss_o, r_g, r_o, w, ora = run_parity("float32", "adagrad", 1, "sigmoid", gather=gather,
                                                 sparse_dw=sparse_dw)
    assert abs(loss_g - loss_o) <= 1e-5 * abs(loss_o), (loss_g, loss_o)
    assert abs(r_g - r_o) <= 1e-5, (r_g, r_o)
    for wg, wo in zip(w[0::2], ora.W):
        assert np.quantile(np.abs(wg - wo), 0.999) < 1e-5
