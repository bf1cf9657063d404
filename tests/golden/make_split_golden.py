"""Generate the preprocessing fixtures by running the REFERENCE split (TrainValidTestSplit.py) here.

Run in the build container only (needs /root/reference):   python tests/golden/make_split_golden.py

What it does
  1. Writes a toy ratings CSV with string ids (the 'amazon' schema: userId, itemId, rating, timestamp;
     string ids avoid the reference's np.int64 JSON failure at TrainValidTestSplit.py:106,115), with
     duplicated (user, item) pairs and a rating of 0.0, to tests/golden/split/ratings.csv.
  2. Loads TrainValidTestSplit.py's functions without its module-level call (the file ends with
     split_data(...) against a hard-coded /data1 path, :222), sets its configuration globals
     (input CSV, output directory, schema 'amazon', include_timestamps False -- the files
     data_reader.py reads -- save_users_and_items True, reverse_user_item_data False / True), seeds
     NumPy's global RNG and calls split_data: the reference's own code writes
     ratingsByUser_dicts_{train,valid,test}.json + unique_{users,items}_list.json (and its MyMediaLite
     CSVs, deleted here) into tests/golden/split/{U,I}/.
  3. The same for numeric-id CSVs of the 'movielens' (float ratings) and 'netflix' (3 columns, integer
     ratings) schemas into tests/golden/split_ml/ and split_nf/ (save_users_and_items False: the
     reference's id-list dump fails on numeric ids).
Only the data (the CSV input and the reference's JSON outputs) is committed; no reference source.
tests/test_preprocess.py checks omnidirectional_collaborative_filtering_amd.preprocess against them.
"""
from __future__ import annotations

import ast
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "split")
REF = "/root/reference/TrainValidTestSplit.py"
SEEDS = {"U": 101, "I": 202}


def write_csv(path, n_users=37, n_items=23, density=0.3, seed=7):
    rng = np.random.RandomState(seed)
    rows = []
    t = 1_000_000
    for u in rng.permutation(n_users):
        for i in rng.permutation(n_items):
            if rng.random_sample() < density:
                t += int(rng.randint(1, 100))
                rows.append(("u%03d" % u, "item_%d" % (7 * i + 3), float(rng.randint(1, 6)), t))
    # the reference's data hazards: a (user, item) pair rated twice, a 0.0 rating
    rows.append((rows[5][0], rows[5][1], 2.0, t + 1))
    rows.append((rows[40][0], rows[40][1], 4.0, t + 2))
    rows.append(("u999", rows[7][1], 0.0, t + 3))
    order = rng.permutation(len(rows))
    with open(path, "w") as f:
        f.write("userId,itemId,rating,timestamp\n")
        for k in order:
            u, i, r, ts = rows[k]
            f.write("%s,%s,%.1f,%d\n" % (u, i, r, ts))
    return len(rows)


def write_numeric_csv(path, schema, n_users=31, n_items=19, density=0.35, seed=11):
    """numeric ids, as the movielens / netflix exports have them: 'movielens' = userId,movieId,rating,timestamp
    with half-star ratings (ml-20m's ratings.csv), 'netflix' = userId,itemId,rating (no timestamp column,
    TrainValidTestSplit.py:64-69) with whole ratings written as floats ("4.0"); plus a duplicated pair and a
    0 rating.  The ratings must parse as floats: with an all-integer frame the reference's pandas rows
    carry np.int64 ids and its json.dump of the dicts fails (:154) -- checked, it raises TypeError."""
    rng = np.random.RandomState(seed)
    rows = []
    t = 900_000_000
    for u in rng.permutation(n_users):
        for i in rng.permutation(n_items):
            if rng.random_sample() < density:
                t += int(rng.randint(1, 100))
                r = rng.randint(1, 11) / 2.0 if schema == "movielens" else float(rng.randint(1, 6))
                rows.append((int(10 * u + 1), int(97 * i + 5), r, t))
    rows.append((rows[3][0], rows[3][1], 3.0, t + 1))
    rows.append((rows[30][0], rows[30][1], 1.0, t + 2))
    rows.append((7777, rows[9][1], 0.0, t + 3))
    order = rng.permutation(len(rows))
    with open(path, "w") as f:
        if schema == "movielens":
            f.write("userId,movieId,rating,timestamp\n")
            for k in order:
                u, i, r, ts = rows[k]
                f.write("%d,%d,%.1f,%d\n" % (u, i, r, ts))
        else:
            f.write("userId,itemId,rating\n")
            for k in order:
                u, i, r, _ = rows[k]
                f.write("%d,%d,%.1f\n" % (u, i, r))
    return len(rows)


def reference_split_functions():
    """TrainValidTestSplit.py's definitions, without its trailing split_data(...) call"""
    with open(REF) as f:
        tree = ast.parse(f.read(), REF)
    tree.body = [n for n in tree.body
                 if not (isinstance(n, ast.Expr) and isinstance(n.value, ast.Call)
                         and getattr(n.value.func, "id", "") == "split_data")]
    ns = {"__name__": "TrainValidTestSplit"}
    exec(compile(tree, REF, "exec"), ns)
    return ns


def main():
    os.makedirs(OUT, exist_ok=True)
    csv = os.path.join(OUT, "ratings.csv")
    n = write_csv(csv)
    meta = {"csv": "ratings.csv", "schema_type": "amazon", "ratings": n, "split": [0.8, 0.1, 0.1], "seeds": SEEDS,
            "generator": "reference TrainValidTestSplit.py split_data via tests/golden/make_split_golden.py"}
    for orient, rev in (("U", False), ("I", True)):
        d = os.path.join(OUT, orient)
        os.makedirs(d, exist_ok=True)
        ns = reference_split_functions()
        ns.update(full_data_filepath=csv, output_filepath=d + "/", schema_type="amazon", build_data_for_omni=True,
                  include_timestamps=False, save_users_and_items=True, reverse_user_item_data=rev)
        np.random.seed(SEEDS[orient])
        ns["split_data"](True)
        for f in ("train_data_mml.csv", "test_data_mml.csv"):
            p = os.path.join(d, f)
            if os.path.exists(p):
                os.remove(p)
        print(orient, sorted(os.listdir(d)))
    with open(os.path.join(OUT, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    # numeric-id schemas: the reference keys rows by str(int(id)) (movielens) / str(id) (netflix) of the
    # pandas row (TrainValidTestSplit.py:124-137; a row of an all-numeric frame is one dtype: float64 with
    # float ratings, so movielens' item ids land in the lists as floats), and has no unique-list dump that
    # works on numeric ids (json.dump of np.int64, :105-118): save_users_and_items False, dicts only
    for schema, sub, seeds in (("movielens", "split_ml", {"U": 303, "I": 404}), ("netflix", "split_nf",
                                                                              {"U": 505, "I": 606})):
        out = os.path.join(HERE, sub)
        os.makedirs(out, exist_ok=True)
        csv = os.path.join(out, "ratings.csv")
        n = write_numeric_csv(csv, schema)
        for orient, rev in (("U", False), ("I", True)):
            d = os.path.join(out, orient)
            os.makedirs(d, exist_ok=True)
            ns = reference_split_functions()
            ns.update(full_data_filepath=csv, output_filepath=d + "/", schema_type=schema, build_data_for_omni=True,
                      include_timestamps=False, save_users_and_items=False, reverse_user_item_data=rev)
            np.random.seed(seeds[orient])
            ns["split_data"](False)
            for f in ("train_data_mml.csv", "test_data_mml.csv"):
                p = os.path.join(d, f)
                if os.path.exists(p):
                    os.remove(p)
            print(schema, orient, sorted(os.listdir(d)))
        with open(os.path.join(out, "meta.json"), "w") as f:
            json.dump({"csv": "ratings.csv", "schema_type": schema, "ratings": n, "split": [0.8, 0.1, 0.1],
                       "seeds": seeds, "save_users_and_items": False,
                       "generator": "reference TrainValidTestSplit.py split_data via tests/golden/make_split_golden.py"},
                      f, indent=1)


if __name__ == "__main__":
    main()
