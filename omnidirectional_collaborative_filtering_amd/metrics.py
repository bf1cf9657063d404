"""The train.py metric set (train.py:102-121) computed from the fused loss-epilogue statistics.

Each batch's masked-MSE epilogue returns SSE, SAE, count_nonzero(y_true + y_pred) and the
per-row SSE; every metric of the reference is a closed form of those (Keras wraps each metric in
a mean over the batch axis, so the per-row sqrt of accurate_RMSE is kept):

  loss / mse           SSE / (b N)
  mean_absolute_error  SAE / (b N)                        ('mae')
  accurate_MAE         SAE B / (b cnt)
  nMAE                 SAE B / (b cnt) / rating_range
  accurate_MSE         SSE B / (b cnt)
  accurate_RMSE        mean over the b rows of sqrt(B * SSE_row / cnt)
where b is the batch's row count and B the script's global batch_size constant the metrics multiply
by (train.py:105,111,116,121: ``MAE*num_items*batch_size``): b = B except for the trailing partial
batch of Keras' Model.fit (train_jester.py:78-79), where the reference's own formulas give these.
The functions below exist so user code can pass them by name exactly as train.py does
(``metrics=['mae', accurate_MAE, nMAE, accurate_RMSE, accurate_MSE]``); calling them on host
arrays evaluates the same closed forms.
"""
from __future__ import annotations

import numpy as np

KNOWN = ("mean_absolute_error", "mean_squared_error", "accurate_MAE", "nMAE", "accurate_RMSE", "accurate_MSE")
ALIASES = {"mae": "mean_absolute_error", "mse": "mean_squared_error"}


def metric_name(m):
    name = m if isinstance(m, str) else getattr(m, "__name__", str(m))
    name = ALIASES.get(name, name)
    if name not in KNOWN:
        raise ValueError("metric %r is not supported by the fused loss epilogue" % (m,))
    return name


def from_stats(name, sse, sae, cnt, row_sse, B, N, rating_range, rows=None):
    b = int(rows) if rows is not None else int(B)
    bN = float(b) * float(N)
    f = float(B) / float(b)
    with np.errstate(divide="ignore", invalid="ignore"):
        if name == "mean_absolute_error":
            return sae / bN
        if name == "mean_squared_error":
            return sse / bN
        if name == "accurate_MAE":
            return np.float64(sae) * f / cnt
        if name == "nMAE":
            return np.float64(sae) * f / cnt / rating_range
        if name == "accurate_MSE":
            return np.float64(sse) * f / cnt
        if name == "accurate_RMSE":
            return float(np.mean(np.sqrt(np.asarray(row_sse[:b], np.float64) * B / cnt)))
    raise ValueError(name)


def _stats(y_true, y_pred):
    y_true = np.asarray(y_true, np.float64)
    y_pred = np.asarray(y_pred, np.float64)
    e = y_pred - y_true
    return float((e * e).sum()), float(np.abs(e).sum()), float(np.count_nonzero(y_true + y_pred)), (e * e).sum(1)


def accurate_MAE(y_true, y_pred):
    sse, sae, cnt, rs = _stats(y_true, y_pred)
    return from_stats("accurate_MAE", sse, sae, cnt, rs, *np.shape(y_true), 1.0)


def accurate_MSE(y_true, y_pred):
    sse, sae, cnt, rs = _stats(y_true, y_pred)
    return from_stats("accurate_MSE", sse, sae, cnt, rs, *np.shape(y_true), 1.0)


def accurate_RMSE(y_true, y_pred):
    sse, sae, cnt, rs = _stats(y_true, y_pred)
    return from_stats("accurate_RMSE", sse, sae, cnt, rs, *np.shape(y_true), 1.0)


def nMAE(y_true, y_pred, rating_range=1.0):
    sse, sae, cnt, rs = _stats(y_true, y_pred)
    return from_stats("nMAE", sse, sae, cnt, rs, *np.shape(y_true), rating_range)


def compute_full_RMSE(sse_total, ratings_count):
    """train.py:243-252: sqrt(sum over test batches of SSE / sum of target_count)."""
    return float(np.sqrt(sse_total / ratings_count))
