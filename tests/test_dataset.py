"""CPU: host rating storage (row-CSR in list order, duplicate chains), the fixed-split semantics of
TrainValidTestSplit.py:74-103, JSON loading against the reference files, and the .npz cache."""
import os

import numpy as np

from omnidirectional_collaborative_filtering_amd.dataset import (FixedSplit, RatingsCSR, dup_chain, load_reference_json,
                                                                 split_ratings, synthetic_ratings)
from oracle.batch_oracle import ReaderOracle

TOY = os.path.join(os.path.dirname(__file__), "golden", "toy")


def test_dup_chain_links_later_duplicates():
    rp = np.array([0, 5, 7])
    col = np.array([3, 1, 3, 2, 3, 4, 4], np.int32)
    d = dup_chain(rp, col)
    assert list(d) == [2, -1, 4, -1, -1, 6, -1]
    assert dup_chain(np.array([0, 2]), np.array([1, 2], np.int32)) is None


def test_from_lists_keeps_list_order_and_none_rows():
    idx = {"a": 0, "b": 1, "c": 2}
    c = RatingsCSR.from_lists(["r1", "r2", "r3"], [[["c", 1.0], ["a", 2.5]], None, [["b", 4.0]]], idx)
    assert list(c.row_ptr) == [0, 2, 2, 3]
    assert list(c.col) == [2, 0, 1]
    assert list(c.val) == [1.0, 2.5, 4.0]


def test_json_loader_matches_reference_reader():
    fs = load_reference_json(TOY, reverse_user_item_data=True)
    ora = ReaderOracle.from_dir(TOY)
    assert fs.train.keys == ora.train_keys
    assert fs.valid_tgt.keys == ora.valid_keys and fs.test_tgt.keys == ora.test_keys
    for i, k in enumerate(ora.train_keys):
        lo, hi = fs.train.row_ptr[i], fs.train.row_ptr[i + 1]
        want = [(ora.col_index[c], v) for c, v in ora.train_dict[k]]
        assert list(zip(fs.train.col[lo:hi], fs.train.val[lo:hi])) == want
    assert fs.train.dup is not None          # the toy data holds one duplicated rating


def test_split_semantics():
    r, c, v = synthetic_ratings(200, 50, 3000, seed=1)
    fs = split_ratings(r, c, v, 200, 50, rng=np.random.RandomState(0))
    n = len(r)
    assert fs.train.nnz == int(n * 0.8)
    assert fs.valid_tgt.nnz == int(n * 0.1)
    assert fs.train.nnz + fs.valid_tgt.nnz + fs.test_tgt.nnz == n
    # valid input row == that row's train ratings; test input == train + valid ratings
    tr_rows = {k: i for i, k in enumerate(fs.train.keys)}
    for i, k in enumerate(fs.valid_in.keys):
        lo, hi = fs.valid_in.row_ptr[i], fs.valid_in.row_ptr[i + 1]
        if k in tr_rows:
            j = tr_rows[k]
            assert sorted(fs.train.col[fs.train.row_ptr[j]:fs.train.row_ptr[j + 1]]) == sorted(fs.valid_in.col[lo:hi])
        else:
            assert hi == lo
    va_rows = {k: i for i, k in enumerate(fs.valid_tgt.keys)}

    def cols(csr, i):
        return list(csr.col[csr.row_ptr[i]:csr.row_ptr[i + 1]])

    for i, k in enumerate(fs.test_in.keys):
        want = (cols(fs.train, tr_rows[k]) if k in tr_rows else []) + \
               (cols(fs.valid_tgt, va_rows[k]) if k in va_rows else [])
        assert sorted(cols(fs.test_in, i)) == sorted(want)


def test_npz_roundtrip(tmp_path):
    fs = load_reference_json(TOY)
    p = str(tmp_path / "d.npz")
    fs.save(p)
    g = FixedSplit.load(p)
    for name in ("train", "valid_in", "valid_tgt", "test_in", "test_tgt"):
        a, b = getattr(fs, name), getattr(g, name)
        assert np.array_equal(a.row_ptr, b.row_ptr) and np.array_equal(a.col, b.col) and np.array_equal(a.val, b.val)


def test_tile_index_segments_match_bruteforce():
    """Column-sorted per-row view used by the masked-MSE row-segment mode: every (row, tile) segment
    holds exactly that row's entries of the tile, with list positions pointing back at them."""
    from omnidirectional_collaborative_filtering_amd.dataset import RatingsCSR
    rng = np.random.RandomState(3)
    n_rows, n_cols = 40, 300
    lists = []
    for r in range(n_rows):
        k = rng.randint(0, 30) if r % 7 else 0
        lists.append([[int(c), float(rng.randint(1, 6))] for c in rng.randint(0, n_cols, size=k)] or None)
    csr = RatingsCSR.from_lists(list(range(n_rows)), lists, {c: c for c in range(n_cols)})
    col_s, val_s, lidx_s, tptr = csr.tile_index(n_cols)
    n_tiles = -(-n_cols // 128)
    assert tptr.shape == (n_rows, n_tiles + 1)
    for r in range(n_rows):
        s0, s1 = csr.row_ptr[r], csr.row_ptr[r + 1]
        for t in range(n_tiles):
            seg = slice(s0 + tptr[r, t], s0 + tptr[r, t + 1])
            want = [(j, csr.col[s0 + j]) for j in range(s1 - s0) if t * 128 <= csr.col[s0 + j] < (t + 1) * 128]
            want.sort(key=lambda z: (z[1], z[0]))
            got = list(zip(lidx_s[seg].tolist(), col_s[seg].tolist()))
            assert got == [(int(j), int(c)) for j, c in want]
            assert np.array_equal(val_s[seg], csr.val[s0 + lidx_s[seg]])
        assert tptr[r, -1] == s1 - s0
