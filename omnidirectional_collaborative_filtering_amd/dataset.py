"""Host-side rating storage: row-CSR in the reference's list order.

The reference keeps ratings as JSON dicts ``row_key -> [[col_raw_id, rating], ...]`` and maps
column ids through ``items_to_densevec`` (data_reader.py:20-28, 85-92).  Here every split is
converted once, at load time, into a row-CSR

    row_ptr int64 [rows+1]   col int32 [nnz] (dense column index)   val float32 [nnz]

whose per-row entry order is the dict's list order (so the j-th NumPy draw of
``choice(..., size=len(list))`` still belongs to the j-th rating, data_reader.py:130-135), plus an
optional duplicate chain (next entry of the same row with the same column) that lets the GPU
scatter reproduce last-write-wins (data_reader.py:158-166).  Fixed-split data (eval_mode
'fixed_split', data_reader.py:57-80) is a train CSR plus (input CSR, target CSR) pairs for valid
and test, rows in target-dict key order.

Also here: the rating-level 80/10/10 split of TrainValidTestSplit.py:74-103 (``split_ratings``), a
synthetic generator shaped like the BASELINE configs, and a binary .npz cache format.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np


def stable_order(major, minor=None):
    """argsort(major * K + minor, kind='stable') for non-negative integer keys, as LSD radix passes
    over 16-bit digits (NumPy's stable sort is a radix sort for 16-bit keys only): O(n) per pass
    instead of an O(n log n) 64-bit merge sort -- the Netflix-sized CSRs (80 M entries) are built in
    seconds, not minutes."""
    keys = [k for k in (minor, major) if k is not None]
    order = None
    for k in keys:
        k = np.asarray(k)
        hi = int(k.max()) if len(k) else 0
        shift = 0
        while True:
            digit = ((k >> shift) & 0xFFFF).astype(np.uint16)
            d = digit if order is None else digit[order]
            o = np.argsort(d, kind="stable")
            order = o if order is None else order[o]
            shift += 16
            if hi >> shift == 0:
                break
    return order


def dup_chain(row_ptr: np.ndarray, col: np.ndarray) -> Optional[np.ndarray]:
    """next[e] = next entry (CSR index) in the same row with the same column, else -1.
    Returns None when the matrix has no duplicate (row, col) pairs."""
    nnz = len(col)
    if nnz == 0:
        return None
    rows = np.repeat(np.arange(len(row_ptr) - 1, dtype=np.int64), np.diff(row_ptr))
    key = rows * (int(col.max()) + 1) + col.astype(np.int64)
    order = stable_order(rows, col.astype(np.int64))
    ks = key[order]
    same = ks[1:] == ks[:-1]
    if not same.any():
        return None
    nxt = np.full(nnz, -1, dtype=np.int32)
    nxt[order[:-1][same]] = order[1:][same].astype(np.int32)
    return nxt


@dataclass
class RatingsCSR:
    row_ptr: np.ndarray
    col: np.ndarray
    val: np.ndarray
    keys: List = field(default_factory=list)
    dup: Optional[np.ndarray] = None
    # column shards (feature parallelism): position of each entry within its full row, and the
    # full rows' lengths (the NumPy reciprocal draws are taken per full row)
    pos: Optional[np.ndarray] = None
    full_lens: Optional[np.ndarray] = None

    @property
    def n_rows(self):
        return len(self.row_ptr) - 1

    @property
    def nnz(self):
        return int(self.row_ptr[-1])

    def row_lengths(self):
        return np.diff(self.row_ptr)

    def rng_lengths(self):
        """entries per row as the reference's RNG sees them (full rows, also for a column shard)"""
        return self.full_lens if self.full_lens is not None else self.row_lengths()

    def tile_index(self, n_cols, tile=128):
        """Column-sorted view for per-tile target lookup (OCF_EPI_MASKED_MSE row-segment mode).

        Returns (col_s, val_s, lidx_s, tptr): the entries of every row sorted by column (stable, so
        duplicates keep list order), each entry's position in the row's list order, and
        tptr[r, t] = number of row-r entries with column < tile*t  (shape [rows, n_tiles + 1])."""
        n_tiles = -(-int(n_cols) // tile)
        lens = self.row_lengths()
        rows = np.repeat(np.arange(self.n_rows, dtype=np.int64), lens)
        order = stable_order(rows, self.col.astype(np.int64))
        col_s = self.col[order]
        val_s = self.val[order]
        lidx_s = (order - self.row_ptr[rows[order]]).astype(np.int32)
        counts = np.bincount(rows * n_tiles + (col_s.astype(np.int64) // tile), minlength=self.n_rows * n_tiles)
        tptr = np.zeros((self.n_rows, n_tiles + 1), dtype=np.int32)
        np.cumsum(counts.reshape(self.n_rows, n_tiles), axis=1, out=tptr[:, 1:])
        return col_s, val_s, lidx_s, tptr

    def column_shard(self, c0, c1):
        """entries with c0 <= col < c1, columns re-based to 0, list order and full-row positions kept"""
        lens = self.row_lengths()
        rows = np.repeat(np.arange(self.n_rows), lens)
        pos = np.arange(self.nnz, dtype=np.int64) - np.repeat(self.row_ptr[:-1], lens)
        if self.pos is not None:
            pos = self.pos.astype(np.int64)
        keep = (self.col >= c0) & (self.col < c1)
        counts = np.bincount(rows[keep], minlength=self.n_rows)
        rp = np.zeros(self.n_rows + 1, dtype=np.int64)
        np.cumsum(counts, out=rp[1:])
        c = RatingsCSR(rp, (self.col[keep] - c0).astype(np.int32), self.val[keep], list(self.keys))
        c.dup = None if self.dup is None else dup_chain(rp, c.col)     # a subset of a dup-free CSR has none
        c.pos = pos[keep].astype(np.int32)
        c.full_lens = self.rng_lengths()
        return c

    @classmethod
    def from_lists(cls, keys, lists, col_index):
        """lists[i] = [[col_raw_id, rating], ...] or None (empty row)."""
        lens = np.fromiter((0 if l is None else len(l) for l in lists), dtype=np.int64, count=len(lists))
        rp = np.zeros(len(lists) + 1, dtype=np.int64)
        np.cumsum(lens, out=rp[1:])
        col = np.empty(int(rp[-1]), dtype=np.int32)
        val = np.empty(int(rp[-1]), dtype=np.float32)
        pos = 0
        for l in lists:
            if l is None:
                continue
            for cid, r in l:
                col[pos] = lookup_col(col_index, cid)
                val[pos] = r
                pos += 1
        c = cls(rp, col, val, list(keys))
        c.dup = dup_chain(rp, col)
        return c

    @classmethod
    def from_coo(cls, rows, cols, vals, n_rows, keys=None, dup_free=False):
        """rows need not be sorted; within a row the given order is kept (stable).  dup_free: the
        caller guarantees unique (row, col) pairs (no duplicate chain to build)."""
        rows = np.asarray(rows, dtype=np.int64)
        order = stable_order(rows)
        counts = np.bincount(rows, minlength=n_rows)
        rp = np.zeros(n_rows + 1, dtype=np.int64)
        np.cumsum(counts, out=rp[1:])
        c = cls(rp, np.asarray(cols, dtype=np.int32)[order], np.asarray(vals, dtype=np.float32)[order],
                list(range(n_rows)) if keys is None else list(keys))
        c.dup = None if dup_free else dup_chain(rp, c.col)
        return c

    def subset_rows(self, idx):
        """Rows idx (negative = empty row) as a new CSR."""
        idx = np.asarray(idx, dtype=np.int64)
        lens = np.where(idx >= 0, self.row_ptr[np.maximum(idx, 0) + 1] - self.row_ptr[np.maximum(idx, 0)], 0)
        rp = np.zeros(len(idx) + 1, dtype=np.int64)
        np.cumsum(lens, out=rp[1:])
        take = np.concatenate([np.arange(self.row_ptr[i], self.row_ptr[i + 1]) for i in idx if i >= 0]) \
            if len(idx) else np.zeros(0, np.int64)
        c = RatingsCSR(rp, self.col[take] if len(take) else np.zeros(0, np.int32),
                       self.val[take] if len(take) else np.zeros(0, np.float32), [])
        c.dup = None if self.dup is None else dup_chain(rp, c.col)     # a subset of a dup-free CSR has none
        return c


def lookup_col(col_index, cid):
    try:
        return col_index[cid]
    except KeyError:
        return col_index[str(cid)]


@dataclass
class FixedSplit:
    """eval_mode='fixed_split' data (data_reader.py:57-80)."""
    num_cols: int
    train: RatingsCSR
    valid_in: RatingsCSR
    valid_tgt: RatingsCSR
    test_in: RatingsCSR
    test_tgt: RatingsCSR
    col_ids: List = field(default_factory=list)

    def column_shard(self, c0, c1):
        """the same split restricted to columns [c0, c1) (feature-parallel rank's slice)"""
        return FixedSplit(c1 - c0, *(getattr(self, k).column_shard(c0, c1)
                                     for k in ("train", "valid_in", "valid_tgt", "test_in", "test_tgt")),
                          col_ids=list(self.col_ids[c0:c1]))

    def save(self, path):
        arrs = {"num_cols": np.array(self.num_cols), "col_ids": np.asarray([str(c) for c in self.col_ids])}
        for name in ("train", "valid_in", "valid_tgt", "test_in", "test_tgt"):
            c = getattr(self, name)
            arrs[name + "/row_ptr"] = c.row_ptr
            arrs[name + "/col"] = c.col
            arrs[name + "/val"] = c.val
            arrs[name + "/keys"] = np.asarray([str(k) for k in c.keys])
        np.savez(path, **arrs)

    @classmethod
    def load(cls, path):
        z = np.load(path, allow_pickle=False)
        parts = {}
        for name in ("train", "valid_in", "valid_tgt", "test_in", "test_tgt"):
            c = RatingsCSR(z[name + "/row_ptr"], z[name + "/col"], z[name + "/val"], list(z[name + "/keys"]))
            c.dup = dup_chain(c.row_ptr, c.col)
            parts[name] = c
        col_ids = list(z["col_ids"]) if "col_ids" in z.files else list(range(int(z["num_cols"])))
        return cls(int(z["num_cols"]), col_ids=col_ids, **parts)


def load_reference_json(filepath, reverse_user_item_data=True, use_json=True):
    """Read the reference's fixed-split files (data_reader.py:20-28, 46-49, 66-80)."""
    if not use_json:
        raise ValueError("pickle inputs are not loaded (unsafe deserialisation); convert to JSON or .npz")

    def rd(name):
        with open(os.path.join(filepath, name + ".json"), "r") as f:
            return json.load(f)

    uniq = rd("unique_users_list" if reverse_user_item_data else "unique_items_list")
    col_index = {c: i for i, c in enumerate(uniq)}
    base = "ratingsByItem" if reverse_user_item_data else "ratingsByUser"
    tr = rd(base + "_dicts_train")
    va_in, va_t = rd(base + "_dicts_valid")
    te_in, te_t = rd(base + "_dicts_test")
    train = RatingsCSR.from_lists(list(tr.keys()), list(tr.values()), col_index)
    vk = list(va_t.keys())
    tk = list(te_t.keys())
    return FixedSplit(
        num_cols=len(uniq),
        train=train,
        valid_in=RatingsCSR.from_lists(vk, [va_in.get(k) for k in vk], col_index),
        valid_tgt=RatingsCSR.from_lists(vk, [va_t[k] for k in vk], col_index),
        test_in=RatingsCSR.from_lists(tk, [te_in.get(k) for k in tk], col_index),
        test_tgt=RatingsCSR.from_lists(tk, [te_t[k] for k in tk], col_index),
        col_ids=list(uniq),
    )


def split_ratings(rows, cols, vals, n_rows, n_cols, split=(0.8, 0.1, 0.1), rng=None, dup_free=False, row_keys=None,
                  col_ids=None):
    """Rating-level permutation split of TrainValidTestSplit.py:74-103, with the reference's orders.

    perm = rng.permutation(n_ratings) (:74; rng = NumPy's global RNG by default, as the reference);
    train / valid / test = perm[:80 %], the next 10 %, the rest (:76-82); test inputs = train + valid
    ratings = perm[:90 %] (:83).  Each split's rows are keyed in the order the reference's
    build_user_item_dict inserts them into its dict -- order of first appearance in that split's
    ratings (:121-149) -- and each row's list keeps the split's rating order; valid / test inputs are
    the target rows' input lists or empty (map_inputs_to_targets, :183-195).  row_keys[r] labels row
    id r (default: the integer itself); col_ids labels the columns (default 0 .. n_cols-1).
    dup_free: the (row, col) pairs are unique (synthetic_ratings), so no split has duplicates.
    """
    rng = np.random if rng is None else rng
    n = len(rows)
    perm = rng.permutation(n)
    ntr, nva = int(n * split[0]), int(n * split[1])
    tr, va, te = perm[:ntr], perm[ntr:ntr + nva], perm[ntr + nva:]
    rows = np.asarray(rows, np.int64)
    cols = np.asarray(cols, np.int32)
    vals = np.asarray(vals, np.float32)
    label = (lambda r: int(r)) if row_keys is None else (lambda r: row_keys[r])

    def by_first_appearance(idx):
        """(CSR of ratings idx keyed by first appearance, row ids in key order, row id -> position or -1)"""
        r = rows[idx]
        uniq, first = np.unique(r, return_index=True)
        order = uniq[np.argsort(first, kind="stable")]
        pos = np.full(n_rows, -1, np.int64)
        pos[order] = np.arange(len(order))
        csr = RatingsCSR.from_coo(pos[r], cols[idx], vals[idx], len(order), keys=[label(x) for x in order],
                                  dup_free=dup_free)
        return csr, order, pos

    train, _, pos_tr = by_first_appearance(tr)
    va_t, order_va, _ = by_first_appearance(va)
    te_t, order_te, _ = by_first_appearance(te)
    te_full, _, pos_te_in = by_first_appearance(perm[:ntr + nva])
    va_in = train.subset_rows(pos_tr[order_va])
    va_in.keys = list(va_t.keys)
    te_in = te_full.subset_rows(pos_te_in[order_te])
    te_in.keys = list(te_t.keys)
    return FixedSplit(n_cols, train, va_in, va_t, te_in, te_t,
                      list(range(n_cols)) if col_ids is None else list(col_ids))


# density / shape table for synthetic inputs (rows x N in I-AutoRec orientation)
SYNTH_SHAPES = {
    "ml100k": dict(rows=1682, cols=943, nnz=100_000, half_stars=False),
    "ml1m": dict(rows=3706, cols=6040, nnz=1_000_209, half_stars=False),
    # BASELINE configs[1] as worded ("256 users x ~3.7k items"): the U orientation, rows = users
    "ml1m_u": dict(rows=6040, cols=3706, nnz=1_000_209, half_stars=False),
    "ml20m": dict(rows=26_744, cols=138_493, nnz=20_000_263, half_stars=True),
    "netflix": dict(rows=17_770, cols=480_189, nnz=100_480_507, half_stars=False),
}


def synthetic_ratings(rows, cols, nnz, half_stars=False, seed=0, skew=0.0):
    """Synthetic ratings, duplicates removed.  skew = 0: uniform rows and columns (multinomial row
    counts); skew = a > 0: row and column popularity both ~ rank^-a over a random permutation (a
    heavy-tailed item / user distribution like the real ratings files: a = 0.5 puts about 0.3 % of
    ML-20M's ratings on its most popular item, as in the real file)."""
    g = np.random.default_rng(seed)
    if skew > 0:
        pr = g.permutation(np.arange(1, rows + 1, dtype=np.float64) ** -skew)
        pc = g.permutation(np.arange(1, cols + 1, dtype=np.float64) ** -skew)
        counts = g.multinomial(nnz, pr / pr.sum())
        counts = np.minimum(counts, cols)
    else:
        counts = g.multinomial(nnz, np.full(rows, 1.0 / rows))
    r = np.repeat(np.arange(rows, dtype=np.int64), counts)
    if skew > 0:
        c = g.choice(cols, size=len(r), p=pc / pc.sum()).astype(np.int64)
    else:
        c = g.integers(0, cols, size=len(r), dtype=np.int64)
    key = np.unique(r * cols + c)
    r = (key // cols).astype(np.int64)
    c = (key % cols).astype(np.int32)
    if half_stars:
        v = g.integers(1, 11, size=len(r)).astype(np.float32) / 2.0
    else:
        v = g.integers(1, 6, size=len(r)).astype(np.float32)
    return r, c, v


def synthetic_fixed_split(name_or_shape, seed=0, scale_rows=None, skew=0.0):
    shp = dict(SYNTH_SHAPES[name_or_shape]) if isinstance(name_or_shape, str) else dict(name_or_shape)
    if scale_rows:
        shp["nnz"] = int(shp["nnz"] * scale_rows / shp["rows"])
        shp["rows"] = scale_rows
    r, c, v = synthetic_ratings(shp["rows"], shp["cols"], shp["nnz"], shp.get("half_stars", False), seed, skew)
    return split_ratings(r, c, v, shp["rows"], shp["cols"], rng=np.random.RandomState(seed), dup_free=True)
