"""CPU: the oracle restatement of data_reader.py is pinned to the reference's own outputs
(tests/golden/batches.npz, produced by importing /root/reference/data_reader.py), and the host half
of the product's epoch plan (permutation + NumPy-exact reciprocal draws) reproduces them too."""
import json
import os

import numpy as np
import pytest

from oracle.batch_oracle import ReaderOracle, reciprocal_cut, scatter_rows_numpy

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOY = os.path.join(GOLD, "toy")


def _cfg():
    with open(os.path.join(GOLD, "batches_config.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLD, "batches.npz"))


@pytest.fixture(scope="module")
def gold_u():
    return np.load(os.path.join(GOLD, _cfg()["u"]["npz"]))


def _drain(gen, n):
    out = [next(gen) for _ in range(n)]
    assert next(gen) is None
    return out


@pytest.mark.parametrize("orient", ["I", "U"])
@pytest.mark.parametrize("ci", range(5))
def test_oracle_reproduces_reference(gold, gold_u, ci, orient):
    """I: ratingsByItem_* + unique_users_list (I-AutoRec); U: ratingsByUser_* + unique_items_list
    (reverse_user_item_data=False, data_reader.py:20-23,46-49)"""
    cfg = _cfg()
    name, sp, pt, aux_type, auxv = cfg["train_configs"][ci]
    B = cfg["B"]
    np.random.seed(cfg["seed_base"] + ci)
    if orient == "U":
        gold = gold_u
        rd = ReaderOracle.from_dir(os.path.join(GOLD, cfg["u"]["dir"]), reverse_user_item_data=False)
    else:
        rd = ReaderOracle.from_dir(TOY)
    seq = [("train1", rd.data_gen(B, sp, "train", True, aux_type, auxv, pass_through=pt), len(rd.train_keys)),
           ("valid", rd.data_gen(B, sp, "valid", True, aux_type, auxv, return_target_count=True), len(rd.valid_keys)),
           ("test", rd.data_gen(B, sp, "test", True, aux_type, auxv, return_target_count=True), len(rd.test_keys)),
           ("train2", rd.data_gen(B, sp, "train", True, aux_type, auxv, pass_through=pt), len(rd.train_keys))]
    for tag, gen, n in seq:
        for bi, item in enumerate(_drain(gen, n // B)):
            for k, a in enumerate(item[0]):
                np.testing.assert_array_equal(a, gold["%s/%s/%d/in%d" % (name, tag, bi, k)])
            np.testing.assert_array_equal(item[1], gold["%s/%s/%d/targets" % (name, tag, bi)])
            if len(item) == 3:
                assert item[2] == int(gold["%s/%s/%d/count" % (name, tag, bi)])


@pytest.mark.parametrize("s", [0.0, 0.123456, 0.3, 0.5, 0.7, 0.9999, 1.0])
def test_choice_restatement(s):
    np.random.seed(7)
    a = np.random.choice([0, 1], size=5000, p=[1 - s, s])
    np.random.seed(7)
    u = np.random.random_sample(5000)
    np.testing.assert_array_equal(a, (u >= reciprocal_cut(s)).astype(int))


def test_uniform_and_stream_concatenation():
    np.random.seed(3)
    x = np.random.uniform(0.2, 0.9, 5)
    y = np.concatenate([np.random.random_sample(4), np.random.random_sample(6)])
    np.random.seed(3)
    assert np.array_equal(x, 0.2 + (0.9 - 0.2) * np.random.random_sample(5))
    assert np.array_equal(y, np.random.random_sample(10))


@pytest.mark.parametrize("orient", ["I", "U"])
@pytest.mark.parametrize("ci", range(5))
def test_product_epoch_plan_matches_reference(gold, gold_u, ci, orient):
    """BatchGenerator.plan (host permutation) + the reciprocal draws of ocf_recip_keep's algorithm (its host
    twin ocf_mt_host_random_sample: the same MT19937 jump-ahead segments, from NumPy's state) + the
    vectorised scatter reproduce the reference train batches."""
    import ctypes

    from omnidirectional_collaborative_filtering_amd import _lib
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    cfg = _cfg()
    name, sp, pt, aux_type, auxv = cfg["train_configs"][ci]
    B = cfg["B"]
    np.random.seed(cfg["seed_base"] + ci)
    if orient == "U":
        gold, meta = gold_u, cfg["u"]["meta"]
        rd = data_reader(meta["num_items"], meta["num_users"], os.path.join(GOLD, cfg["u"]["dir"]),
                         eval_mode="fixed_split", reverse_user_item_data=False)
    else:
        meta = cfg["meta"]
        rd = data_reader(meta["num_users"], meta["num_items"], TOY, eval_mode="fixed_split",
                         reverse_user_item_data=True)
    gen = rd.data_gen(B, sp, "train", True, aux_type, auxv, pass_through_input_training=pt)
    tr = rd.data.train
    rows, boff, _ = gen.plan(tr.row_lengths())
    st = np.random.get_state()
    key = np.ascontiguousarray(st[1], dtype=np.uint32).copy()
    pos = ctypes.c_int32(int(st[2]))
    n = len(rows) * B + int(boff[:, -1].sum())
    u = np.empty(n, np.float64)
    _lib.call("ocf_mt_host_random_sample", key.ctypes.data, ctypes.addressof(pos), n, u.ctypes.data)
    d = 0
    for bi in range(len(rows)):
        s = sp[0] + (sp[1] - sp[0]) * u[d:d + B]                             # data_reader.py:120
        ue = u[d + B: d + B + int(boff[bi, -1])]                              # :130, row after row
        d += B + int(boff[bi, -1])
        kb = ue >= np.repeat((1.0 - s) / ((1.0 - s) + s), np.diff(boff[bi]))
        m_in, m_out, x, t, m_miss = scatter_rows_numpy(tr.row_ptr, tr.col, tr.val, rows[bi], rd.num_items, keep=kb,
                                                       aux=auxv, pass_through=pt)
        np.testing.assert_array_equal(x, gold["%s/train1/%d/in0" % (name, bi)])
        np.testing.assert_array_equal(t, gold["%s/train1/%d/targets" % (name, bi)])
        out_mask = gold["%s/train1/%d/in%d" % (name, bi, 1 if aux_type is None else 2)]
        np.testing.assert_array_equal(m_out, out_mask)
