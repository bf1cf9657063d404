"""Ratings CSV -> fixed split (the reference's offline preprocessing, TrainValidTestSplit.py:31-119,
121-195), as a FixedSplit (.npz cache) and/or the JSON files data_reader.py reads.

    python -m omnidirectional_collaborative_filtering_amd.preprocess ratings.csv --schema movielens \\
        [--reverse] [--seed S] [--out data.npz] [--json DIR]

Same semantics as split_data: the CSV's columns are named by schema (:39-69; 'netflix' has no
timestamp); with reverse_user_item_data the first two columns swap roles (I-AutoRec rows = items); a
rating-level permutation from NumPy's global RNG (:74; --seed seeds it first) splits 80/10/10
(:76-83); every split's rows are keyed in dict-insertion order (first appearance in that split's
ratings, build_user_item_dict :121-149) with the row keys as strings (movielens: str(int(id)),
:127; the others str(id)), lists in rating order; valid inputs = the row's train list, test inputs =
its train + valid list, or none (map_inputs_to_targets :183-195).  Columns are the other id in order
of first appearance in the CSV (the reference's unique_*_list, :106-118).  Ids are what the
reference's pandas row holds (:125): in an all-numeric CSV with float ratings every id is a float
(list ids 1193.0; netflix row keys '6.0'), with string ids they stay strings.  (An all-integer CSV --
integer ratings too -- makes the reference's json.dump fail on np.int64 ids, :154; here it works, ids
as ints.)

Differences that are deliberate: the JSON writer names the files the way data_reader.py reads them
(ratingsByItem_* + unique_users_list for I-AutoRec; the reference's split writes ratingsByUser_*
either way) and writes the id lists whatever the id type (the reference's json.dump
of np.int64 ids fails, :106,115); MyMediaLite CSVs (:213-219) and timestamps are not produced
(timestamps are out of scope, data_reader.py:358-359).
"""
from __future__ import annotations

import argparse
import json
import os

import numpy as np

from .dataset import FixedSplit, split_ratings

SCHEMAS = {"movielens": 4, "amazon": 4, "beeradvocate": 4, "yelp": 4, "netflix": 3}


def _row_scalar(df):
    """What the reference's ``ratings.iloc[i]`` makes of one id (TrainValidTestSplit.py:125): a row of a frame
    whose columns are all numeric is a single-dtype Series (np.result_type of the columns -- float64 as soon
    as the ratings are floats), so numeric ids come out as floats (movielens item ids land in the lists as
    1193.0, netflix row keys as '6.0'); a frame with a string column gives an object row (ids unchanged)."""
    kinds = [np.dtype(d) for d in df.dtypes]
    if all(k.kind in "iuf" for k in kinds):
        common = np.result_type(*kinds)
        return float if common.kind == "f" else int
    return lambda x: _plain(x)


def _key(schema, scalar=lambda x: x):
    """the row key the reference's build_user_item_dict writes (TrainValidTestSplit.py:126-135)"""
    if schema == "movielens":
        return lambda x: str(int(scalar(x)))
    return lambda x: str(scalar(x))


def _plain(v):
    """JSON-serialisable scalar for an id (NumPy scalars -> Python)"""
    return v.item() if isinstance(v, np.generic) else v


def split_csv(path, schema="movielens", reverse_user_item_data=False, split=(0.8, 0.1, 0.1), rng=None):
    """TrainValidTestSplit.split_data on the ratings CSV at `path` -> FixedSplit (rows keyed by the
    reference's dict keys, columns labelled by the other id)."""
    import pandas as pd
    if schema not in SCHEMAS:
        raise ValueError("schema must be one of %s" % sorted(SCHEMAS))
    df = pd.read_csv(path)
    if df.shape[1] != SCHEMAS[schema]:
        raise ValueError("schema %r expects %d columns, the CSV has %d" % (schema, SCHEMAS[schema], df.shape[1]))
    row_raw = df.iloc[:, 1 if reverse_user_item_data else 0].to_numpy()
    col_raw = df.iloc[:, 0 if reverse_user_item_data else 1].to_numpy()
    vals = df.iloc[:, 2].to_numpy(dtype=np.float64)
    row_codes, row_uniq = pd.factorize(row_raw, sort=False)
    col_codes, col_uniq = pd.factorize(col_raw, sort=False)          # first appearance = pd.unique order
    scalar = _row_scalar(df)
    key = _key(schema, scalar)
    row_keys = [key(x) for x in row_uniq]
    col_ids = [scalar(_plain(x)) for x in col_uniq]                  # the ids the reference's lists carry
    return split_ratings(row_codes.astype(np.int64), col_codes.astype(np.int32), vals.astype(np.float32),
                         len(row_uniq), len(col_uniq), split=split, rng=rng, row_keys=row_keys, col_ids=col_ids)


def _lists(csr, col_ids):
    out = {}
    for i, k in enumerate(csr.keys):
        lo, hi = int(csr.row_ptr[i]), int(csr.row_ptr[i + 1])
        out[str(k)] = [[col_ids[int(c)], float(v)] for c, v in zip(csr.col[lo:hi], csr.val[lo:hi])]
    return out


def save_reference_json(fs, dirpath, reverse_user_item_data=False):
    """The fixed-split files data_reader.py:20-28,46-80 loads (use_json=True), named for the orientation
    it is opened with."""
    os.makedirs(dirpath, exist_ok=True)
    base = "ratingsByItem" if reverse_user_item_data else "ratingsByUser"
    cols = "unique_users_list" if reverse_user_item_data else "unique_items_list"
    ids = [_plain(c) for c in fs.col_ids]

    def with_none(inp, tgt):
        d = _lists(inp, ids)
        return {str(k): (d[str(k)] or None) for k in tgt.keys}

    files = {base + "_dicts_train": _lists(fs.train, ids),
             base + "_dicts_valid": [with_none(fs.valid_in, fs.valid_tgt), _lists(fs.valid_tgt, ids)],
             base + "_dicts_test": [with_none(fs.test_in, fs.test_tgt), _lists(fs.test_tgt, ids)],
             cols: ids}
    for name, obj in files.items():
        with open(os.path.join(dirpath, name + ".json"), "w") as f:
            json.dump(obj, f)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("csv")
    ap.add_argument("--schema", default="movielens", choices=sorted(SCHEMAS))
    ap.add_argument("--reverse", action="store_true", help="reverse_user_item_data (I-AutoRec: rows are items)")
    ap.add_argument("--seed", type=int, default=None, help="np.random.seed before the split (default: unseeded)")
    ap.add_argument("--out", default=None, help="FixedSplit .npz cache (data_reader(..., dataset=path))")
    ap.add_argument("--json", default=None, help="directory for the reference-layout JSON files")
    a = ap.parse_args(argv)
    if a.seed is not None:
        np.random.seed(a.seed)
    fs = split_csv(a.csv, a.schema, a.reverse)
    if a.out:
        fs.save(a.out)
    if a.json:
        save_reference_json(fs, a.json, a.reverse)
    print(json.dumps({"rows_train": fs.train.n_rows, "rows_valid": fs.valid_tgt.n_rows, "rows_test": fs.test_tgt.n_rows,
                      "columns": fs.num_cols, "ratings": int(fs.train.nnz + fs.valid_tgt.nnz + fs.test_tgt.nnz)}))
    return fs


if __name__ == "__main__":
    main()
