"""CPU: the range-ordered row-gather tables (data_reader BatchGenerator._range_chunk_tables, OcfGatherArgs perm /
ch_slot) -- every batch row's entries covered exactly once in its column-sorted view, a row's slots contiguous
and in entry order (row_cptr), the chunks dispatched range by range, and the sorted view a permutation of the
rating lists."""
import numpy as np
import torch

from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings


def test_range_chunk_tables_cover_rows():
    rows, cols = 300, 2000
    r, c, v = synthetic_ratings(rows, cols, 60000, half_stars=True, seed=4, skew=0.8)
    data = split_ratings(r, c, v, rows, cols, rng=np.random.RandomState(4))
    rd = data_reader(cols, rows, dataset=data, eval_mode="fixed_split", rng="device", device=torch.device("cpu"))
    R = 7
    rd.gather_ranges = R
    gen = rd.data_gen(64, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
    gen._start()
    ch = gen.chunks1
    src = gen.src1.host
    sv = ch["sorted"]
    col_s, perm = sv["col"].numpy(), sv["perm"].numpy()
    for row in range(src.n_rows):
        a, b = src.row_ptr[row], src.row_ptr[row + 1]
        assert (np.diff(col_s[a:b]) >= 0).all()
        assert sorted(perm[a:b].tolist()) == list(range(b - a))
        assert (src.col[a + perm[a:b]] == col_s[a:b]).all()
    ch_row, j0, j1 = ch["ch_row"].numpy(), ch["ch_j0"].numpy(), ch["ch_j1"].numpy()
    cptr = ch["row_cptr"].numpy()
    bounds = np.arange(R + 1) * cols // R
    multi = 0
    for bi in range(gen.num_batches):
        c0, c1 = int(ch["cbase"][bi]), int(ch["cbase"][bi + 1])
        b = ch_row[c0:c1] & 4095
        slot = ch_row[c0:c1] >> 12
        j0b, j1b = j0[c0:c1], j1[c0:c1]
        assert sorted(slot.tolist()) == list(range(c1 - c0))
        rng_of = []
        for k in range(c1 - c0):
            row = gen.rows_host[bi][b[k]]
            s = src.row_ptr[row]
            rng_of.append(int(np.searchsorted(bounds, col_s[s + j0b[k]], side="right")) - 1)
            assert (col_s[s + j0b[k]:s + j1b[k]] >= bounds[rng_of[-1]]).all()
            assert (col_s[s + j0b[k]:s + j1b[k]] < bounds[rng_of[-1] + 1]).all()
        assert (np.diff(rng_of) >= 0).all(), "chunks dispatched range by range"
        for bb in range(gen.B):
            mine = np.flatnonzero(b == bb)
            order = mine[np.argsort(slot[mine])]
            assert slot[order].tolist() == list(range(cptr[bi][bb], cptr[bi][bb + 1]))
            row = gen.rows_host[bi][bb]
            n = src.row_ptr[row + 1] - src.row_ptr[row] if row >= 0 else 0
            if len(order):
                assert j0b[order[0]] == 0 and j1b[order[-1]] == n
                assert (j0b[order[1:]] == j1b[order[:-1]]).all()
                assert (j1b[order] - j0b[order] <= 256).all() and (j1b[order] > j0b[order]).all()
            else:
                assert n == 0
            multi += len(order) > R
    assert multi > 0          # some rows have more chunks than ranges (a range over 64 entries)
