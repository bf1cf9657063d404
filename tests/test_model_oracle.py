"""CPU: internal consistency of the NumPy model oracle (its gradients vs finite differences, the
optimizer equations, the metric closed forms).  The oracle is the checker for the GPU parity tests."""
import numpy as np
import pytest

from oracle.model_oracle import (AdagradOracle, AdamOracle, OmniOracle, RMSpropOracle, batch_metrics,
                                 compute_full_RMSE)


def _problem(seed=0, B=6, N=9, H=(5,), k=1, act="sigmoid", dropout=None, l2=None):
    rng = np.random.RandomState(seed)
    x = rng.rand(B, k * N) * (rng.rand(B, k * N) < 0.4)
    m = -1.0 * (rng.rand(B, N) < 0.5)
    t = np.where(m != 0, rng.randint(1, 11, size=(B, N)) / 2.0, 0.0)
    ora = OmniOracle([k * N] + list(H) + [N], activation=act, dropout=dropout, l2=l2).init(seed)
    ora.W = [w.astype(np.float64) for w in ora.W]
    ora.b = [rng.randn(*b.shape) * 0.1 for b in ora.b]
    drop = None
    if dropout:
        drop = [(rng.rand(B, h) >= dropout).astype(np.float64) for h in H]
    return ora, x, m, t, drop


@pytest.mark.parametrize("act", ["sigmoid", "tanh", "relu"])
@pytest.mark.parametrize("H", [(5,), (4, 3)])
@pytest.mark.parametrize("dropout,l2", [(None, None), (0.3, None), (None, 0.01)])
def test_oracle_gradients_finite_difference(act, H, dropout, l2):
    ora, x, m, t, drop = _problem(act=act, H=H, dropout=dropout, l2=l2)
    loss, _, gW, gb = ora.loss_and_grads(x, m, t, drop)
    eps = 1e-6
    for li in range(len(ora.W)):
        for arr, g in ((ora.W[li], gW[li]), (ora.b[li], gb[li])):
            flat = arr.reshape(-1)
            for idx in np.random.RandomState(li).choice(flat.size, min(6, flat.size), replace=False):
                old = flat[idx]
                flat[idx] = old + eps
                lp = ora.loss_and_grads(x, m, t, drop)[0]
                flat[idx] = old - eps
                lm = ora.loss_and_grads(x, m, t, drop)[0]
                flat[idx] = old
                num = (lp - lm) / (2 * eps)
                assert abs(num - g.reshape(-1)[idx]) < 1e-6 + 1e-5 * abs(num)


def test_mse_is_sse_over_BN():
    ora, x, m, t, _ = _problem()
    loss, y, _, _ = ora.loss_and_grads(x, m, t)
    assert np.isclose(loss, ((y - t) ** 2).sum() / t.size)


def test_optimizer_equations():
    p = [np.array([1.0, -2.0, 0.5])]
    g = [np.array([0.1, -0.3, 0.0])]
    a = AdagradOracle(lr=0.01, epsilon=1e-8)
    out = a.step(p, g)[0]
    np.testing.assert_allclose(out, p[0] - 0.01 * g[0] / (np.abs(g[0]) + 1e-8))
    r = RMSpropOracle(lr=0.001, rho=0.9)
    out = r.step(p, g)[0]
    acc = 0.1 * g[0] ** 2
    np.testing.assert_allclose(out, p[0] - 0.001 * g[0] / (np.sqrt(acc) + 1e-8))
    ad = AdamOracle(lr=0.001)
    out = ad.step(p, g)[0]
    lr_t = 0.001 * np.sqrt(1 - 0.999) / (1 - 0.9)
    mt, vt = 0.1 * g[0], 0.001 * g[0] ** 2
    np.testing.assert_allclose(out, p[0] - lr_t * mt / (np.sqrt(vt) + 1e-8))


def test_metrics_closed_forms():
    from omnidirectional_collaborative_filtering_amd import metrics as M
    rng = np.random.RandomState(1)
    B, N = 7, 11
    t = np.where(rng.rand(B, N) < 0.3, rng.randint(1, 6, (B, N)).astype(float), 0.0)
    y = np.where(t != 0, -rng.rand(B, N) * 5, 0.0)
    ref = batch_metrics(t, y, N, B, 4.0)
    e = y - t
    sse, sae, cnt = (e * e).sum(), np.abs(e).sum(), np.count_nonzero(t + y)
    rs = (e * e).sum(1)
    assert np.isclose(M.from_stats("accurate_MSE", sse, sae, cnt, rs, B, N, 4.0), ref["accurate_MSE"])
    assert np.isclose(M.from_stats("accurate_MAE", sse, sae, cnt, rs, B, N, 4.0), ref["accurate_MAE"])
    assert np.isclose(M.from_stats("nMAE", sse, sae, cnt, rs, B, N, 4.0), ref["nMAE"])
    assert np.isclose(M.from_stats("accurate_RMSE", sse, sae, cnt, rs, B, N, 4.0), ref["accurate_RMSE"])
    assert np.isclose(M.from_stats("mean_absolute_error", sse, sae, cnt, rs, B, N, 4.0), ref["mean_absolute_error"])
    assert np.isclose(compute_full_RMSE([y], [t], cnt), np.sqrt(sse / cnt))
    # Keras' trailing partial batch of Model.fit (b = 4 rows; the metrics still multiply by the script's
    # batch_size constant B, train.py:105-121): the per-batch values the reference's formulas give
    b = 4
    ref = batch_metrics(t[:b], y[:b], N, B, 4.0)
    e = e[:b]
    sse, sae, cnt = (e * e).sum(), np.abs(e).sum(), np.count_nonzero(t[:b] + y[:b])
    rs = np.concatenate([(e * e).sum(1), np.zeros(B - b)])      # the padding rows carry nothing
    for name in ("accurate_MSE", "accurate_MAE", "nMAE", "accurate_RMSE", "mean_absolute_error"):
        assert np.isclose(M.from_stats(name, sse, sae, cnt, rs, B, N, 4.0, rows=b), ref[name]), name
    assert np.isclose(M.from_stats("mean_squared_error", sse, sae, cnt, rs, B, N, 4.0, rows=b), ref["loss"])


@pytest.mark.parametrize("dropout", [None, 0.2])
@pytest.mark.parametrize("act", ["sigmoid", "tanh"])
def test_sparse_restatement_equals_dense(dropout, act):
    """OmniOracle.loss_and_grads_sparse (the ML-20M / Netflix-width form) is the dense oracle on the
    same batch: loss, gradients and the rounding envelope agree to fp64 roundoff"""
    import scipy.sparse as sp
    rng = np.random.RandomState(3)
    B, N, H = 12, 57, 7
    pat = rng.rand(B, N) < 0.15
    t = np.where(pat, rng.randint(1, 11, size=(B, N)) / 2.0, 0.0)
    m = -1.0 * pat
    ora = OmniOracle([N, H, N], activation=act, dropout=dropout).init(1)
    ora.W = [w.astype(np.float64) for w in ora.W]
    ora.b = [rng.randn(*b.shape) * 0.1 for b in ora.b]
    drop = [(rng.rand(B, H) >= dropout).astype(np.float64)] if dropout else None
    loss, _, gW, gb = ora.loss_and_grads(t, m, t, drop)
    GW, Gb = ora.grad_magnitudes(t, m, t, drop, u=2.0 ** -11)
    X = sp.csr_matrix(t)
    M = sp.csr_matrix(m)
    ls, _, sW, sb, sGW, sGb = ora.loss_and_grads_sparse(X, M, X, drop, u=2.0 ** -11, chunk=5)
    assert abs(ls - loss) <= 1e-13 * abs(loss)
    for a, b in zip(gW + gb + GW + Gb, sW + sb + sGW + sGb):
        np.testing.assert_allclose(np.asarray(b), a, rtol=1e-11, atol=1e-16)
    h = ora.forward_hidden_sparse(X)
    y, _ = ora.forward(t, m)
    np.testing.assert_allclose(-(h @ ora.W[1] + ora.b[1]) * pat, y, rtol=1e-12, atol=1e-15)
