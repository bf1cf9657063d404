"""NumPy restatement of the reference's model / loss / optimizer / metric arithmetic.
TEST INFRASTRUCTURE ONLY.  PARITY UNPINNED (see oracle/__init__.py).

The reference builds its graph with Keras 2.0.4 on TF 1.3 (README.md:17-24), neither of which
exists in this image, and it ships no tests.  This module restates the published Keras 2.0.4
equations for exactly the graph model.py builds:

  model.py:43-60   inputs; x = concat([data, observed_mask?, second_mask?])   (last axis)
  model.py:64-73   L x [ h = act(x W + b) ; Dropout(p, noise_shape=[B, H]) ]
  model.py:81-86   y_full = h W_out + b_out (linear) ; y = output_mask * y_full
  model.py:66,82   optional l2(lambda) kernel regulariser  -> loss += lambda * sum(W^2)
  train.py:49      'mean_squared_error' -> mean over last axis, then mean over batch = SSE / (B N)
  train.py:50-51   Adagrad(lr, epsilon, decay=0)     Keras 2.0.4 Adagrad.get_updates
  train_jester.py:61 'rmsprop' (lr 1e-3, rho 0.9, eps 1e-8)  Keras 2.0.4 RMSprop.get_updates
  north_star       Adam (lr 1e-3, b1 .9, b2 .999, eps 1e-8)   Keras 2.0.4 Adam.get_updates
  train.py:102-121 mae / accurate_MAE / nMAE / accurate_RMSE / accurate_MSE
  train.py:243-255 compute_full_RMSE
Weights use Keras' (in, out) layout; glorot_uniform init U(+-sqrt(6/(fan_in+fan_out))), zero bias.
"""
from __future__ import annotations

import numpy as np


def act_fwd(name, z):
    if name == "sigmoid":
        return 1.0 / (1.0 + np.exp(-z))
    if name == "tanh":
        return np.tanh(z)
    if name == "relu":
        return np.maximum(z, 0)
    if name == "linear":
        return z
    raise ValueError(name)


def act_grad_from_out(name, a, z):
    if name == "sigmoid":
        return a * (1.0 - a)
    if name == "tanh":
        return 1.0 - a * a
    if name == "relu":
        return (z > 0).astype(a.dtype)
    if name == "linear":
        return np.ones_like(a)
    raise ValueError(name)


def glorot_uniform(rng, fan_in, fan_out, dtype=np.float32):
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=(fan_in, fan_out)).astype(dtype)


class OmniOracle:
    """Parameters: ``self.W[i]`` (in, out), ``self.b[i]`` (out,), i = 0..L (L hidden + output)."""

    def __init__(self, dims, activation="sigmoid", dropout=None, l2=None, dtype=np.float64):
        self.dims = list(dims)
        self.activation = activation
        self.dropout = dropout
        self.l2 = l2
        self.dtype = dtype
        self.W = []
        self.b = []

    def init(self, seed):
        rng = np.random.RandomState(seed)
        self.W = [glorot_uniform(rng, i, o).astype(self.dtype) for i, o in zip(self.dims[:-1], self.dims[1:])]
        self.b = [np.zeros(o, self.dtype) for o in self.dims[1:]]
        return self

    def set_params(self, W, b):
        self.W = [np.array(w, dtype=self.dtype) for w in W]
        self.b = [np.array(x, dtype=self.dtype) for x in b]
        return self

    # ---- forward: model.py:43-99 -----------------------------------------------------
    def forward(self, x_in, out_mask, drop_masks=None):
        """x_in: the concatenated layer-0 input [B, d0]; drop_masks: list of {0,1} [B, H] or None."""
        dt = self.dtype
        hs = [np.asarray(x_in, dt)]
        zs = []
        L = len(self.W) - 1
        for i in range(L):
            z = hs[-1] @ self.W[i] + self.b[i]
            a = act_fwd(self.activation, z)
            if drop_masks is not None and drop_masks[i] is not None:
                keep = 1.0 - self.dropout
                a = a * (np.asarray(drop_masks[i], dt) / dt(keep))
            zs.append(z)
            hs.append(a)
        y_full = hs[-1] @ self.W[L] + self.b[L]
        y = np.asarray(out_mask, dt) * y_full
        return y, (hs, zs, y_full)

    # ---- loss + backward (Keras MSE + l2) -------------------------------------------
    def loss_and_grads(self, x_in, out_mask, targets, drop_masks=None):
        dt = self.dtype
        y, (hs, zs, _) = self.forward(x_in, out_mask, drop_masks)
        T = np.asarray(targets, dt)
        Bn, N = T.shape
        e = y - T
        loss = np.sum(e * e) / dt(Bn * N)
        if self.l2 is not None:
            loss = loss + sum(self.l2 * np.sum(w * w) for w in self.W)
        g = (2.0 / (Bn * N)) * e * np.asarray(out_mask, dt)          # dL/dy_full
        L = len(self.W) - 1
        gW = [None] * (L + 1)
        gb = [None] * (L + 1)
        gW[L] = hs[L].T @ g
        gb[L] = g.sum(0)
        d = g @ self.W[L].T
        for i in range(L - 1, -1, -1):
            if drop_masks is not None and drop_masks[i] is not None:
                d = d * (np.asarray(drop_masks[i], dt) / dt(1.0 - self.dropout))
                a_pre = act_fwd(self.activation, zs[i])
            else:
                a_pre = hs[i + 1]
            d = d * act_grad_from_out(self.activation, a_pre, zs[i])
            gW[i] = hs[i].T @ d
            gb[i] = d.sum(0)
            if i > 0:
                d = d @ self.W[i].T
        if self.l2 is not None:
            gW = [gw + 2.0 * self.l2 * w for gw, w in zip(gW, self.W)]
        return loss, y, gW, gb

    # ---- rounding-error envelope of the gradient (parity tolerances for 16-bit MFMA operands) ----
    def grad_magnitudes(self, x_in, out_mask, targets, drop_masks=None, u=2.0 ** -11):
        """Per-element magnitude sums of the gradient computation, for a running-error bound: the same
        backward pass as loss_and_grads with every product replaced by its absolute value, started
        from |y - t| + u * (|h| |W_out| + |b_out|) (a 16-bit operand rounds y by ~u of that magnitude,
        which the residual y - t does not shrink).  A kernel whose operands are rounded to unit
        roundoff u (f16: 2^-11, bf16: 2^-8) computes gradient element g_i within ~c * u * G_i of the
        exact one, c = the number of roundings along the chain.  Returns (GW, Gb) shaped like (gW, gb).
        Adagrad parity tests scale their per-element tolerance by G_i / |g_i| (the update's
        g / sqrt(sum g^2) is ill-conditioned exactly where that ratio is large)."""
        dt = self.dtype
        _, (hs, zs, y_full) = self.forward(x_in, out_mask, drop_masks)
        T = np.asarray(targets, dt)
        M = np.asarray(out_mask, dt)
        Bn, N = T.shape
        L = len(self.W) - 1
        ymag = np.abs(hs[L]) @ np.abs(self.W[L]) + np.abs(self.b[L])
        g = (2.0 / (Bn * N)) * (np.abs(M * y_full - T) + u * ymag) * np.abs(M)
        GW = [None] * (L + 1)
        Gb = [None] * (L + 1)
        GW[L] = np.abs(hs[L]).T @ g
        Gb[L] = g.sum(0)
        d = g @ np.abs(self.W[L]).T
        for i in range(L - 1, -1, -1):
            a_pre = act_fwd(self.activation, zs[i])
            if drop_masks is not None and drop_masks[i] is not None:
                d = d * (np.asarray(drop_masks[i], dt) / dt(1.0 - self.dropout))
            d = d * np.abs(act_grad_from_out(self.activation, a_pre, zs[i]))
            GW[i] = np.abs(hs[i]).T @ d
            Gb[i] = d.sum(0)
            if i > 0:
                d = d @ np.abs(self.W[i]).T
        return GW, Gb

    def forward_hidden_sparse(self, X):
        """hidden activations (inference: no dropout) of one hidden layer for a scipy CSR input"""
        return act_fwd(self.activation, np.asarray(X @ self.W[0]) + self.b[0])

    # ---- the same equations on sparse batches (ML-20M / Netflix sizes) ---------------------------
    def loss_and_grads_sparse(self, X, out_mask, T, drop_masks=None, u=None, chunk=1 << 17):
        """loss_and_grads for one hidden layer with the batch held sparse: X, out_mask, T are scipy
        CSR [B, N] (out_mask / T share one sparsity pattern: the rating entries; model.py:81-86 makes
        y zero everywhere else, so the unobserved (0 - 0)^2 terms of Keras' MSE add nothing and their
        gradient is exactly zero).  Mathematically identical to loss_and_grads on the densified
        arrays (checked on CPU in tests/test_model_oracle.py); the dense [B, N] arrays never exist, so
        ML-20M (N = 138,493) and Netflix (N = 480,189) batches fit.  With u, also returns the
        grad_magnitudes envelope (GW, Gb).  Returns loss, (entry rows, cols, y), gW, gb[, GW, Gb]."""
        import scipy.sparse as sp
        assert len(self.W) == 2, "sparse restatement: one hidden layer"
        dt = self.dtype
        Bn, N = T.shape
        M = out_mask.tocsr()
        Tm = T.tocsr()
        z = np.asarray(X @ self.W[0]) + self.b[0]
        a = act_fwd(self.activation, z)
        h = a
        if drop_masks is not None and drop_masks[0] is not None:
            h = a * (np.asarray(drop_masks[0], dt) / dt(1.0 - self.dropout))
        coo = M.tocoo()
        r, c, m = coo.row, coo.col, coo.data.astype(dt)
        if not (np.array_equal(M.indptr, Tm.indptr) and np.array_equal(M.indices, Tm.indices)):
            raise ValueError("out_mask and targets must share one sparsity pattern (the rating entries)")
        t = Tm.data.astype(dt)
        W1 = self.W[1]
        yf = np.empty(len(r), dt)
        ymag = np.empty(len(r), dt) if u is not None else None
        for s in range(0, len(r), chunk):
            rr, cc = r[s:s + chunk], c[s:s + chunk]
            yf[s:s + chunk] = np.einsum("ij,ji->i", h[rr], W1[:, cc]) + self.b[1][cc]
            if u is not None:
                ymag[s:s + chunk] = np.einsum("ij,ji->i", np.abs(h[rr]), np.abs(W1[:, cc])) + np.abs(self.b[1][cc])
        y = m * yf
        e = y - t
        loss = float(np.sum(e * e) / dt(Bn * N))
        G = sp.csr_matrix(((2.0 / (Bn * N)) * e * m, (r, c)), shape=(Bn, N))
        gW1 = np.asarray((G.T @ h).T)                  # (H, N) = h^T G
        gb1 = np.asarray(G.sum(0)).ravel()
        d = np.asarray(G @ W1.T)                       # [B, H]
        if drop_masks is not None and drop_masks[0] is not None:
            d = d * (np.asarray(drop_masks[0], dt) / dt(1.0 - self.dropout))
        sg = act_grad_from_out(self.activation, a, z)
        d = d * sg
        gW0 = np.asarray(X.T @ d)
        gb0 = d.sum(0)
        out = [loss, (r, c, y), [gW0, gW1], [gb0, gb1]]
        if u is not None:
            Ga = sp.csr_matrix(((2.0 / (Bn * N)) * (np.abs(e) + u * ymag) * np.abs(m), (r, c)), shape=(Bn, N))
            GW1 = np.asarray((Ga.T @ np.abs(h)).T)
            Gb1 = np.asarray(Ga.sum(0)).ravel()
            da = np.asarray(Ga @ np.abs(W1).T)
            if drop_masks is not None and drop_masks[0] is not None:
                da = da * (np.asarray(drop_masks[0], dt) / dt(1.0 - self.dropout))
            da = da * np.abs(sg)
            Xa = X.copy()
            Xa.data = np.abs(Xa.data)
            out += [[np.asarray(Xa.T @ da), GW1], [da.sum(0), Gb1]]
        return tuple(out)

    def params(self):
        out = []
        for w, b in zip(self.W, self.b):
            out += [w, b]
        return out

    def set_flat(self, flat):
        self.W = flat[0::2]
        self.b = flat[1::2]


# ---- optimizers (Keras 2.0.4 get_updates; accumulators start at 0) ------------------
class AdagradOracle:
    def __init__(self, lr=0.01, epsilon=1e-8, decay=0.0):
        self.lr, self.eps, self.decay = lr, epsilon, decay
        self.acc = None
        self.iterations = 0

    def step(self, params, grads):
        if self.acc is None:
            self.acc = [np.zeros_like(p) for p in params]
        lr = self.lr
        if self.decay > 0:
            lr = lr * (1.0 / (1.0 + self.decay * self.iterations))
        out = []
        for i, (p, g) in enumerate(zip(params, grads)):
            a = self.acc[i] + g * g
            self.acc[i] = a
            out.append(p - lr * g / (np.sqrt(a) + self.eps))
        self.iterations += 1
        return out


class RMSpropOracle:
    def __init__(self, lr=0.001, rho=0.9, epsilon=1e-8, decay=0.0):
        self.lr, self.rho, self.eps, self.decay = lr, rho, epsilon, decay
        self.acc = None
        self.iterations = 0

    def step(self, params, grads):
        if self.acc is None:
            self.acc = [np.zeros_like(p) for p in params]
        lr = self.lr
        if self.decay > 0:
            lr = lr * (1.0 / (1.0 + self.decay * self.iterations))
        out = []
        for i, (p, g) in enumerate(zip(params, grads)):
            a = self.rho * self.acc[i] + (1.0 - self.rho) * g * g
            self.acc[i] = a
            out.append(p - lr * g / (np.sqrt(a) + self.eps))
        self.iterations += 1
        return out


class AdamOracle:
    def __init__(self, lr=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-8, decay=0.0):
        self.lr, self.b1, self.b2, self.eps, self.decay = lr, beta_1, beta_2, epsilon, decay
        self.m = None
        self.v = None
        self.iterations = 0

    def step(self, params, grads):
        if self.m is None:
            self.m = [np.zeros_like(p) for p in params]
            self.v = [np.zeros_like(p) for p in params]
        lr = self.lr
        if self.decay > 0:
            lr = lr * (1.0 / (1.0 + self.decay * self.iterations))
        t = self.iterations + 1
        lr_t = lr * (np.sqrt(1.0 - self.b2 ** t) / (1.0 - self.b1 ** t))
        out = []
        for i, (p, g) in enumerate(zip(params, grads)):
            m = self.b1 * self.m[i] + (1.0 - self.b1) * g
            v = self.b2 * self.v[i] + (1.0 - self.b2) * g * g
            self.m[i], self.v[i] = m, v
            out.append(p - lr_t * m / (np.sqrt(v) + self.eps))
        self.iterations += 1
        return out


# ---- metrics: train.py:102-121 (Keras wraps each in a mean over the batch axis) ---------
def batch_metrics(y_true, y_pred, num_items, batch_size, rating_range):
    y_true = np.asarray(y_true, np.float64)
    y_pred = np.asarray(y_pred, np.float64)
    Bn, N = y_true.shape
    e = y_pred - y_true
    mae_rows = np.abs(e).mean(axis=1)          # metrics.mae  -> [B]
    mse_rows = (e * e).mean(axis=1)            # metrics.mse  -> [B]
    n_pred = float(np.count_nonzero(y_true + y_pred))
    scale = num_items * batch_size / n_pred if n_pred > 0 else np.inf
    return {
        "loss": float(mse_rows.mean()),
        "mean_absolute_error": float(mae_rows.mean()),
        "accurate_MAE": float((mae_rows * scale).mean()),
        "nMAE": float((mae_rows * scale).mean() / rating_range),
        "accurate_RMSE": float(np.sqrt(mse_rows * scale).mean()),
        "accurate_MSE": float((mse_rows * scale).mean()),
    }


def compute_full_RMSE(predictions, targets, ratings_count):
    """train.py:243-252."""
    sse = 0.0
    for p, t in zip(predictions, targets):
        d = np.asarray(p, np.float64) - np.asarray(t, np.float64)
        sse += float(np.sum(d * d))
    return np.sqrt(sse / ratings_count)
