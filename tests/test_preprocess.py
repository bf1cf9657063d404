"""CPU: the CSV -> fixed-split preprocessing against the REFERENCE's own split (TrainValidTestSplit.py
run on tests/golden/split/ratings.csv by tests/golden/make_split_golden.py, both orientations, string
ids, a duplicated pair and a 0.0 rating): same row keys in the same order, same lists in the same order,
same column ids, for train, valid inputs / targets and test inputs / targets; then the JSON writer and the
.npz cache round-trip, and the CLI runs."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from omnidirectional_collaborative_filtering_amd.dataset import FixedSplit, load_reference_json
from omnidirectional_collaborative_filtering_amd.preprocess import save_reference_json, split_csv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPLIT = os.path.join(ROOT, "tests", "golden", "split")
PARTS = ("train", "valid_in", "valid_tgt", "test_in", "test_tgt")


def _meta():
    with open(os.path.join(SPLIT, "meta.json")) as f:
        return json.load(f)


def _same(a, b):
    assert a.num_cols == b.num_cols
    assert [str(c) for c in a.col_ids] == [str(c) for c in b.col_ids]
    for p in PARTS:
        x, y = getattr(a, p), getattr(b, p)
        assert [str(k) for k in x.keys] == [str(k) for k in y.keys], p
        np.testing.assert_array_equal(x.row_ptr, y.row_ptr, err_msg=p)
        np.testing.assert_array_equal(x.col, y.col, err_msg=p)
        np.testing.assert_array_equal(x.val, y.val, err_msg=p)


@pytest.mark.parametrize("orient", ["U", "I"])
def test_split_matches_reference_split(orient):
    meta = _meta()
    np.random.seed(meta["seeds"][orient])
    fs = split_csv(os.path.join(SPLIT, meta["csv"]), meta["schema_type"], reverse_user_item_data=orient == "I")
    # the reference writes ratingsByUser_* + unique_items_list (= the column ids) in both orientations
    ref = load_reference_json(os.path.join(SPLIT, orient), reverse_user_item_data=False)
    _same(fs, ref)
    assert fs.train.dup is not None            # the duplicated (user, item) pair stayed in train
    assert (fs.train.val == 0.0).any() or (fs.test_tgt.val == 0.0).any() or (fs.valid_tgt.val == 0.0).any()


@pytest.mark.parametrize("orient", ["U", "I"])
def test_json_writer_and_npz_roundtrip(tmp_path, orient):
    meta = _meta()
    np.random.seed(meta["seeds"][orient])
    rev = orient == "I"
    fs = split_csv(os.path.join(SPLIT, meta["csv"]), meta["schema_type"], reverse_user_item_data=rev)
    save_reference_json(fs, str(tmp_path / "j"), reverse_user_item_data=rev)
    _same(load_reference_json(str(tmp_path / "j"), reverse_user_item_data=rev), fs)
    fs.save(str(tmp_path / "d.npz"))
    _same(FixedSplit.load(str(tmp_path / "d.npz")), fs)


def test_cli(tmp_path):
    meta = _meta()
    out = subprocess.run([sys.executable, "-m", "omnidirectional_collaborative_filtering_amd.preprocess",
                          os.path.join(SPLIT, meta["csv"]), "--schema", meta["schema_type"], "--seed",
                          str(meta["seeds"]["I"]), "--reverse", "--out", str(tmp_path / "d.npz"), "--json",
                          str(tmp_path / "j")], cwd=ROOT, capture_output=True, text=True, check=True)
    info = json.loads(out.stdout.strip().splitlines()[-1])
    assert info["ratings"] == meta["ratings"]
    ref = load_reference_json(os.path.join(SPLIT, "I"), reverse_user_item_data=False)
    _same(FixedSplit.load(str(tmp_path / "d.npz")), ref)
    _same(load_reference_json(str(tmp_path / "j"), reverse_user_item_data=True), ref)


def _ref_dicts(d):
    out = {}
    for part in ("train", "valid", "test"):
        with open(os.path.join(d, "ratingsByUser_dicts_%s.json" % part)) as f:
            out[part] = json.load(f)
    return out


def _same_json(a, b):
    """equal JSON structures with the same key order and the same id types (float ids stay floats)"""
    if isinstance(a, dict):
        assert isinstance(b, dict) and list(a) == list(b)
        for k in a:
            _same_json(a[k], b[k])
    elif isinstance(a, list):
        assert isinstance(b, list) and len(a) == len(b)
        for x, y in zip(a, b):
            _same_json(x, y)
    else:
        assert a == b and type(a) is type(b), (a, b)


@pytest.mark.parametrize("sub", ["split_ml", "split_nf"])
@pytest.mark.parametrize("orient", ["U", "I"])
def test_numeric_schemas_match_reference(tmp_path, sub, orient):
    """'movielens' (row keys str(int(id)), :127) and 'netflix' (3 columns, :64-69; keys str(id) of the float
    row, e.g. '31.0') on numeric-id CSVs, against the reference's own split of the same CSV (make_split_golden
    .py; save_users_and_items False): the JSON files save_reference_json writes equal the reference's -- same
    row keys in the same order, the same lists in the same order, item ids as the floats the reference writes"""
    d = os.path.join(ROOT, "tests", "golden", sub)
    with open(os.path.join(d, "meta.json")) as f:
        meta = json.load(f)
    rev = orient == "I"
    np.random.seed(meta["seeds"][orient])
    fs = split_csv(os.path.join(d, meta["csv"]), meta["schema_type"], reverse_user_item_data=rev)
    save_reference_json(fs, str(tmp_path / "j"), reverse_user_item_data=rev)
    ours = {}
    base = "ratingsByItem" if rev else "ratingsByUser"
    for part in ("train", "valid", "test"):
        with open(str(tmp_path / "j" / ("%s_dicts_%s.json" % (base, part)))) as f:
            ours[part] = json.load(f)
    ref = _ref_dicts(os.path.join(d, orient))
    _same_json(ref, ours)
    ids = [e[0] for lst in ref["train"].values() for e in lst]
    assert all(isinstance(i, float) for i in ids)      # the reference's float ids (all-numeric float frame)
    if meta["schema_type"] == "netflix":
        assert all(k.endswith(".0") for k in ref["train"])
    # ... and data_reader reads them back (float ids find their columns in the id list)
    fs2 = load_reference_json(str(tmp_path / "j"), reverse_user_item_data=rev)
    _same(fs2, fs)
