"""Restatement of the reference's dense-batch assembly (TEST INFRASTRUCTURE ONLY).

Follows /root/reference/data_reader.py:
  * id map                        data_reader.py:20-28   (column index = position in unique list)
  * set sizes / orders            data_reader.py:72-80   (train = train-dict keys, valid/test = target-dict keys)
  * build_sparse_batch            data_reader.py:95-200  (dense, no timestamps)
  * build_sparse_batch_fixed_split data_reader.py:202-298 (dense, no timestamps)
  * data_gen                      data_reader.py:314-419

RNG: the reference draws from NumPy's *global* legacy RandomState.  Per batch it calls
``uniform(s0, s1, B)`` (data_reader.py:120) and then, per row, ``choice([0,1], n, p=[1-s,s])``
(:130).  Both are restated on ``random_sample``:
    uniform(a, b, n)            == a + (b - a) * random_sample(n)
    choice([0,1], n, p=[1-s,s]) == (random_sample(n) >= c0),  c0 = (1-s) / ((1-s) + s)
(verified numerically against NumPy 2.2 for s in {0, .123456, .3, .5, .7, .9999, 1}).
Consecutive ``random_sample`` calls concatenate, so one call per batch for all rows is the same stream.

Two implementations:
  ``ReaderOracle``           per-rating Python loops in the reference's order (small cases; also
                             the scalar CPU baseline in bench.py)
  ``scatter_rows_numpy``     vectorised NumPy scatter with the same last-write-wins semantics
"""
from __future__ import annotations

import json
import os

import numpy as np


def reciprocal_cut(s):
    """Threshold c0 such that ``choice([0,1], p=[1-s, s])`` returns 1 iff ``u >= c0``.

    NumPy builds ``cdf = cumsum([1-s, s]); cdf /= cdf[-1]`` and returns ``searchsorted(cdf, u, 'right')``.
    """
    s = float(s)
    return (1.0 - s) / ((1.0 - s) + s)


def load_reference_json(dirpath, fname):
    with open(os.path.join(dirpath, fname + ".json"), "r") as f:
        return json.load(f)


class ReaderOracle:
    """Pure-Python restatement of ``data_reader`` for eval_mode='fixed_split' (and ablation train)."""

    def __init__(self, unique_cols, train_dict, valid_pair=None, test_pair=None):
        # data_reader.py:24-28 -- column id -> dense index, in unique-list order
        self.col_index = {}
        for i, c in enumerate(unique_cols):
            self.col_index[c] = i
        self.num_cols = len(unique_cols)
        self.train_dict = train_dict
        self.valid_pair = valid_pair
        self.test_pair = test_pair
        # data_reader.py:73-80 (keys() lists; py3 insertion order == JSON order)
        self.train_keys = list(train_dict.keys())
        self.valid_keys = list(valid_pair[1].keys()) if valid_pair is not None else []
        self.test_keys = list(test_pair[1].keys()) if test_pair is not None else []

    @classmethod
    def from_dir(cls, dirpath, reverse_user_item_data=True):
        base = "ratingsByItem" if reverse_user_item_data else "ratingsByUser"
        uniq = load_reference_json(dirpath, "unique_users_list" if reverse_user_item_data else "unique_items_list")
        tr = load_reference_json(dirpath, base + "_dicts_train")
        va = load_reference_json(dirpath, base + "_dicts_valid")
        te = load_reference_json(dirpath, base + "_dicts_test")
        return cls(uniq, tr, va, te)

    # ---- data_reader.py:95-200 -------------------------------------------------------
    def train_batch(self, order, B, start, s_range, aux, pass_through):
        N = self.num_cols
        m_in = np.zeros((B, N))
        x = np.zeros((B, N))
        m_miss = np.zeros((B, N))
        t = np.zeros((B, N))
        m_out = np.zeros((B, N))
        s_rows = s_range[0] + (s_range[1] - s_range[0]) * np.random.random_sample(B)   # :120
        for r in range(B):
            key = order[start + r]
            entries = self.train_dict[key]                                              # :128
            draws = np.random.random_sample(len(entries))                               # :130
            keep = draws >= reciprocal_cut(s_rows[r])
            for j, (cid, rating) in enumerate(entries):
                c = self.col_index[cid]
                if keep[j]:                                                             # :158-163
                    m_in[r, c] = aux
                    x[r, c] = rating
                    if pass_through:
                        m_out[r, c] = aux
                        t[r, c] = rating
                else:                                                                   # :164-166
                    m_out[r, c] = aux
                    t[r, c] = rating
                m_miss[r, c] = aux                                                      # :169
        return m_in, m_out, x, t, m_miss

    # ---- data_reader.py:202-298 ------------------------------------------------------
    def eval_batch(self, pair, order, B, start, aux):
        inp, tgt = pair
        N = self.num_cols
        m_in = np.zeros((B, N))
        x = np.zeros((B, N))
        m_miss = np.zeros((B, N))
        t = np.zeros((B, N))
        m_out = np.zeros((B, N))
        count = 0
        for r in range(B):
            key = order[start + r]
            if inp[key] is not None:                                                    # :234-252
                for cid, rating in inp[key]:
                    c = self.col_index[cid]
                    m_in[r, c] = aux
                    x[r, c] = rating
                    m_miss[r, c] = aux
            for cid, rating in tgt[key]:                                                # :256-268
                c = self.col_index[cid]
                m_out[r, c] = aux
                t[r, c] = rating
                m_miss[r, c] = aux
                count += 1
        return m_in, m_out, x, t, m_miss, count

    # ---- data_reader.py:314-419 ------------------------------------------------------
    def data_gen(self, B, s_range, split="train", shuffle=True, aux_type="dropout", aux=-1,
                 return_target_count=False, pass_through=False):
        keys = {"train": self.train_keys, "valid": self.valid_keys, "test": self.test_keys}[split]
        order = np.random.permutation(keys) if shuffle else keys                       # :326-327
        for b in range(len(keys) // B):                                                 # :329
            if split == "train":
                m_in, m_out, x, t, m_miss = self.train_batch(order, B, b * B, s_range, aux, pass_through)
                count = None
            else:
                pair = self.valid_pair if split == "valid" else self.test_pair
                m_in, m_out, x, t, m_miss, count = self.eval_batch(pair, order, B, b * B, aux)
            inputs = assemble_input_list(aux_type, x, m_in, m_out, m_miss)
            if split != "train" and return_target_count:
                yield inputs, t, count
            else:
                yield inputs, t
        while True:                                                                     # :418-419
            yield None


def assemble_input_list(aux_type, x, m_in, m_out, m_miss):
    """Model-input list order of data_reader.py:341-361 / :389-411 (no timestamps)."""
    if aux_type is None:
        return [x, m_out]
    if aux_type == "causal":
        feed = m_miss
    elif aux_type in ("dropout", "both"):
        feed = m_in
    elif aux_type == "zeros":
        feed = np.zeros_like(m_in)
    else:
        raise ValueError("unknown auxilliary_mask_type %r" % (aux_type,))
    out = [x, feed, m_out]
    if aux_type == "both":
        out.append(m_miss)
    return out


def scatter_rows_numpy(row_ptr, col, val, rows, N, keep=None, aux=-1.0, pass_through=True, dtype=np.float64):
    """Vectorised restatement of the dense scatter for rows ``rows`` of a CSR matrix.

    ``keep`` (per entry of the gathered rows, in CSR order) marks input ratings (reciprocal split);
    None means all kept.  Duplicate (row, col) entries resolve last-write-wins in list order
    (data_reader.py:158-166), which NumPy fancy assignment reproduces (later index wins).
    Returns m_in, m_out, x, t, m_miss.
    """
    B = len(rows)
    starts = row_ptr[rows]
    ends = row_ptr[np.asarray(rows) + 1]
    lens = ends - starts
    idx = np.concatenate([np.arange(s, e) for s, e in zip(starts, ends)]) if B else np.zeros(0, np.int64)
    r = np.repeat(np.arange(B), lens)
    c = col[idx]
    v = val[idx].astype(np.float64)
    if keep is None:
        keep = np.ones(len(idx), dtype=bool)
    keep = np.asarray(keep, dtype=bool)
    m_in = np.zeros((B, N), dtype)
    x = np.zeros((B, N), dtype)
    m_out = np.zeros((B, N), dtype)
    t = np.zeros((B, N), dtype)
    m_miss = np.zeros((B, N), dtype)
    ki = np.nonzero(keep)[0]
    di = np.nonzero(~keep)[0]
    m_in[r[ki], c[ki]] = aux
    x[r[ki], c[ki]] = v[ki]
    tgt = np.arange(len(idx)) if pass_through else di
    # targets: written by kept entries (pass-through) and by dropped entries, in list order
    m_out[r[tgt], c[tgt]] = aux
    t[r[tgt], c[tgt]] = v[tgt]
    m_miss[r, c] = aux
    return m_in, m_out, x, t, m_miss


def train_batch_loop_csr(row_ptr, col, val, rows, N, s_range=(1.0, 1.0), aux=-1.0, pass_through=True):
    """build_sparse_batch (data_reader.py:95-200) over a CSR instead of dicts: same float64 zeros,
    same per-batch uniform and per-row choice draws, same per-rating scalar stores.  This is the
    scalar CPU baseline bench.py times (one core)."""
    B = len(rows)
    m_in = np.zeros([B, N])
    x = np.zeros([B, N])
    m_miss = np.zeros([B, N])
    t = np.zeros([B, N])
    m_out = np.zeros([B, N])
    s_rows = np.random.uniform(low=s_range[0], high=s_range[1], size=B)
    for r in range(B):
        lo, hi = int(row_ptr[rows[r]]), int(row_ptr[rows[r] + 1])
        split = np.random.choice([0, 1], size=hi - lo, p=[1 - s_rows[r], s_rows[r]])
        for j in range(lo, hi):
            c = col[j]
            v = val[j]
            if split[j - lo] == 1:
                m_in[r, c] = aux
                x[r, c] = v
                if pass_through:
                    m_out[r, c] = aux
                    t[r, c] = v
            else:
                m_out[r, c] = aux
                t[r, c] = v
            m_miss[r, c] = aux
    return m_in, m_out, x, t, m_miss
