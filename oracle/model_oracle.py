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
